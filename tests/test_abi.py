"""The C-ABI library loads (no GPU needed) and exports every function that
include/*.h declares; the oracle is not linked into it."""
import ctypes
import os
import re
import subprocess

from conftest import ROOT

LIB = os.path.join(ROOT, "pairphone_amd", "libmelpe_amd.so")


def declared_functions():
    names = set()
    for h in ("melpe.h", "melpe_batch.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*\b([a-z_0-9]+)\s*\(", src, re.M):
            names.add(m.group(1))
    return names


def test_declared_symbols_exported():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(LIB)
    names = declared_functions()
    assert {"melpe_i", "melpe_a", "melpe_s", "melpe_n", "melpe_engine_create",
            "melpe_encode_dev", "melpe_decode_dev"} <= names
    for n in sorted(names):
        assert hasattr(lib, n), "missing export " + n


def test_no_oracle_in_product():
    out = subprocess.run(["nm", "-D", LIB], capture_output=True, text=True).stdout
    # reference symbols (its global names) must not be in the product
    for bad in ("melp_ana_init", "melp_syn_init", "ref_add", "quant_par", "hpspeech"):
        assert re.search(r"\b%s\b" % bad, out) is None, bad
    deps = subprocess.run(["ldd", LIB], capture_output=True, text=True).stdout
    assert "hostemu" not in deps and "ref_" not in deps


def test_codec_kernels_have_no_flat_accesses():
    """the build-time guard (pairphone_amd/build.py check_no_flat): the
    codec kernels reach private memory only through scratch_ instructions,
    never generic flat_ ones (the FLAT aperture fault, kern.h)"""
    from pairphone_amd.build import check_no_flat, device_disassembly
    objdir = os.path.join(ROOT, "build", "obj", "libmelpe_amd")
    assert os.path.isdir(objdir), "run __graft_entry__.build() first"
    check_no_flat(objdir)
    dis = device_disassembly(os.path.join(objdir, "k_ana.o"))
    assert any("k_enc_ana" in k for k in dis)
