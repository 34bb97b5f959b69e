# round 6: the pipelined encode (next superframe's NPP beside the analysis)
# against the serialised step, 262,144 and 65,536 channels
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06j && mkdir -p $O && export TMPDIR=/tmp &&
MELPE_AMD_LIB=build/var/pipe.so timeout -k 10 400 python3 -u tools/pipe_exp.py 262144 10 2 > $O/pipe_262k.json 2> $O/pipe_262k.err &&
MELPE_AMD_LIB=build/var/pipe.so timeout -k 10 300 python3 -u tools/pipe_exp.py 65536 10 2 > $O/pipe_65k.json 2> $O/pipe_65k.err
