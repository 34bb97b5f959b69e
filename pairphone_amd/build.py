"""Build recipe of the engine (called by __graft_entry__.build()).

1. When the reference is present (the dev container, never the GPU box):
   compile it into oracle/_ref/ (oracle/Makefile) and refresh the table blob
   (oracle/dump_tables.py).  Both are the checker side, not the product.
2. Compile the HIP engine for gfx950 into pairphone_amd/libmelpe_amd.so
   (hipcc; the tables are embedded with .incbin).
3. Compile the host-emulation build of the same device sources
   (build/libmelpe_hostemu.so, g++) used by the CPU-side tests to check the
   kernel logic against the reference without a GPU.  The product library
   never loads it.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pairphone_amd", "csrc")
LIB = os.path.join(ROOT, "pairphone_amd", "libmelpe_amd.so")
EMU = os.path.join(ROOT, "build", "libmelpe_hostemu.so")
REF = "/root/reference/melpe"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# the offload target (MELPE_ARCH for A/B builds, e.g. gfx950:xnack-)
ARCH = os.environ.get("MELPE_ARCH", "gfx950")


def _run(cmd, **kw):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, **kw)


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _sources():
    out = []
    for d in (CSRC, os.path.join(ROOT, "include")):
        for f in os.listdir(d):
            if f.endswith((".h", ".hip", ".cpp")):
                out.append(os.path.join(d, f))
    out.append(os.path.join(ROOT, "pairphone_amd", "data", "melpe_tables.bin"))
    return out


def build_oracle():
    if not os.path.isdir(REF):
        print("reference not present: using prebuilt oracle/_ref and committed tables")
        return
    _run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "-j8"])
    _run([sys.executable, os.path.join(ROOT, "oracle", "dump_tables.py")])


PROF_LIB = os.path.join(ROOT, "pairphone_amd", "libmelpe_amd_prof.so")


TUS = ("engine", "k_npp", "k_ana", "k_ana_mw", "k_harm", "k_dec", "k_r24")
# the codec TUs compile their whole call tree inline, so every access to a
# lane's private state is a scratch_/global_ instruction with counted waits
# instead of a generic FLAT access; this is what costs compile
# time, hence one TU per kernel, compiled in parallel
HOT_TUS = ("k_npp", "k_ana", "k_ana_mw", "k_harm", "k_dec", "k_r24")
# per-TU code-generation options, each kept by an A/B on MI355X: the lane
# analysis without the scheduler's unclustered high-register-pressure
# rescheduling stage, 25.54-25.56 -> 25.38-25.40 ms at 262,144 channels
# (profiles/r06_sch_flags_ab.txt)
TU_FLAGS = {"k_ana": ["-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule"]}


def build_engine(force=False, prof=False, defs=(), out=None, tus_defs=None, hot=HOT_TUS, only=None):
    """hipcc build of the product library (prof=True: the stage-timer
    diagnostics variant libmelpe_amd_prof.so, -DMELPE_PROF); only=(tu, ...)
    recompiles just those TUs and relinks with the other TUs' objects from
    the previous build (a development shortcut; the default rebuilds all)"""
    out = out or (PROF_LIB if prof else LIB)
    deps = _sources()
    if not force and not _newer(out, deps):
        return out
    blob = os.path.join(ROOT, "pairphone_amd", "data", "melpe_tables.bin")
    tag = os.path.splitext(os.path.basename(out))[0]
    objdir = os.path.join(ROOT, "build", "obj", tag)
    os.makedirs(objdir, exist_ok=True)
    common = [HIPCC, "-O3", "--offload-arch=" + ARCH, "-std=c++17", "-fPIC", "-c",
              "-Wno-unused-result", "-Wno-unused-value", '-DMELPE_TABLES_BIN="%s"' % blob] \
        + (["-DMELPE_PROF"] if prof else []) + ["-D" + d for d in defs] \
        + os.environ.get("MELPE_EXTRA_FLAGS", "").split()
    procs, objs = [], []
    for tu in TUS:
        o = os.path.join(objdir, tu + ".o")
        objs.append(o)
        if only is not None and tu not in only and os.path.exists(o):
            continue
        extra = (["-DMELPE_INLINE_ALL"] if tu in hot else []) + TU_FLAGS.get(tu, [])
        if tus_defs and tu in tus_defs:
            extra += ["-D" + d for d in tus_defs[tu]]
        cmd = common + extra + [os.path.join(CSRC, tu + ".hip"), "-o", o]
        print("+", " ".join(cmd), flush=True)
        procs.append((tu, subprocess.Popen(cmd)))
    bad = [tu for tu, p in procs if p.wait() != 0]
    if bad:
        raise RuntimeError("hipcc failed for " + ", ".join(bad))
    check_no_flat(objdir)
    tmp = out + ".tmp"
    _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC"] + objs + ["-o", tmp])
    os.replace(tmp, out)
    return out


LLVM_BIN = "/opt/rocm/lib/llvm/bin"


def device_disassembly(obj, arch=None):
    """gfx950 disassembly of one hipcc object (its offload bundle), as
    {kernel symbol: [instruction lines]}"""
    arch = arch or ARCH
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:
        fat, elf = os.path.join(tmp, "fat.bin"), os.path.join(tmp, "dev.elf")
        subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=" + fat, obj], check=True)
        for a in dict.fromkeys((arch, "gfx950")):	# an A/B build may mix targets
            r = subprocess.run([os.path.join(LLVM_BIN, "clang-offload-bundler"), "--unbundle", "--type=o",
                                "--input=" + fat, "--targets=hipv4-amdgcn-amd-amdhsa--" + a,
                                "--output=" + elf], capture_output=True)
            if r.returncode == 0 and os.path.getsize(elf) > 0:
                break
        else:
            raise RuntimeError("no gfx950 code object in " + obj)
        txt = subprocess.run([os.path.join(LLVM_BIN, "llvm-objdump"), "-d", "--no-show-raw-insn",
                              elf], check=True, capture_output=True, text=True).stdout
    out, cur = {}, None
    for line in txt.splitlines():
        if line.endswith(">:") and "<" in line:
            cur = line[line.index("<") + 1:-2]
            out[cur] = []
        elif cur and line.startswith("\t"):
            out[cur].append(line.strip())
    return out


# codec kernels that must not contain generic (FLAT) accesses: a FLAT access
# to the private segment is aperture-checked before its offset is added,
# which faulted on gfx950 (kern.h FLAT_GUARD_BYTES)
NO_FLAT = ("k_enc_ana", "k_enc_harm", "k_enc_tail", "k_decode", "k_vad", "k_enc_npp", "k_npp",
           "k_demodulate", "k_enc24",
           "k_dec24", "k_helpers_eval")


def check_no_flat(objdir):
    bad = []
    for f in sorted(os.listdir(objdir)):
        if not f.endswith(".o"):
            continue
        for sym, ins in device_disassembly(os.path.join(objdir, f)).items():
            if any(k in sym for k in NO_FLAT):
                n = sum(1 for i in ins if i.startswith("flat_"))
                if n:
                    bad.append("%s: %d flat_ instructions" % (sym, n))
    if bad:
        raise RuntimeError("generic FLAT accesses in codec kernels: " + "; ".join(bad))


def build_hostemu(force=False):
    deps = _sources()
    if not force and not _newer(EMU, deps):
        return EMU
    os.makedirs(os.path.dirname(EMU), exist_ok=True)
    tmp = EMU + ".tmp"
    _run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I" + CSRC,
          os.path.join(CSRC, "hostemu.cpp"), "-o", tmp])
    os.replace(tmp, EMU)
    return EMU


def build_opcount(force=False):
    """host build with the basic-op census compiled in (tools/opcount.py)"""
    out = os.path.join(ROOT, "build", "libmelpe_opcount.so")
    if not force and not _newer(out, _sources()):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    _run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-DMELPE_OPCOUNT", "-I" + CSRC,
          os.path.join(CSRC, "hostemu.cpp"), "-o", out + ".tmp"])
    os.replace(out + ".tmp", out)
    return out


DROPIN = os.path.join(ROOT, "build", "dropin")


def build_dropin(force=False):
    """The reference's own callers of melpe.h -- melpe/encoder.c,
    melpe/decoder.c and melpe_dec.c, compiled unchanged where they lie --
    linked against libmelpe_amd.so instead of the reference's libmelpe.a
    (INTEGRATION.md §1).  Test infrastructure: tests/test_dropin.py runs them
    on the GPU box.  Only where the reference sources exist; the binaries
    travel with the tree."""
    if not os.path.isdir(REF):
        return
    os.makedirs(DROPIN, exist_ok=True)
    srcs = {"encoder": os.path.join(REF, "encoder.c"), "decoder": os.path.join(REF, "decoder.c"),
            "melpe_dec": os.path.join(os.path.dirname(REF), "melpe_dec.c")}
    for name, src in srcs.items():
        out = os.path.join(DROPIN, name)
        if not force and not _newer(out, [src, LIB]):
            continue
        # -include: our include/melpe.h is seen first; the reference header the
        # source includes itself then only repeats the same prototypes
        _run(["gcc", "-O2", "-w", "-include", os.path.join(ROOT, "include", "melpe.h"), src,
              "-L" + os.path.dirname(LIB), "-lmelpe_amd", "-Wl,-rpath-link,/opt/rocm/lib",
              "-Wl,-rpath,$ORIGIN/../../pairphone_amd", "-o", out])


def build_all(force=False):
    build_oracle()
    build_engine(force)
    build_dropin(force)
    if os.path.exists(os.path.join(CSRC, "hostemu.cpp")):
        build_hostemu(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
