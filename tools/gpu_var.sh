# A/B of engine variants (build/var/*.so) against the default build: encode
# parity tests per variant, then a short bench line each.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline" &&
timeout -k 10 300 python $B > gpurun_out/v_base.json 2> gpurun_out/v_base.err &&
for v in "$@"; do
  MELPE_AMD_LIB=build/var/$v.so timeout -k 10 300 python -u -m pytest ${VAR_TESTS:-tests/test_encode.py} -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_$v.log 2>&1 &&
  MELPE_AMD_LIB=build/var/$v.so timeout -k 10 300 python $B > gpurun_out/v_$v.json 2> gpurun_out/v_$v.err || exit 1
done
