"""Basic-op parity: ops.h (the device basic-op library, compiled for the
host) against the reference's own compiled operators (oracle/_ref/
libref_ops.so built from melpe/mathhalf_i.h, melpe/mathdp31.c).
Exhaustive over int16 x shift in [-40, 40]; int16 x (every 7th int16) for
add/sub/mult/L_mult/divide_s; 1M randomised 32/40-bit cases with edge values.
"""
import os
import subprocess

from conftest import ROOT, REF_DIR


def test_basic_ops_match_reference(tmp_path, ref_tool):
    exe = str(tmp_path / "ops_check")
    subprocess.run(["g++", "-O2", "-I" + os.path.join(ROOT, "pairphone_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "ops_check.cpp"),
                    "-L" + REF_DIR, "-lref_ops", "-Wl,-rpath," + REF_DIR, "-o", exe],
                   check=True)
    out = subprocess.run([exe, "1000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "OK 0 mismatches" in out.stdout
