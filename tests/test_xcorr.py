"""The exact packed-pair correlators (dsp.h xcorr_pairs / magsq_pairs,
analysis.h fp_sums9) -- the v_dot2_i32_i16 paths that replace saturating
L_mac chains once a chain is proved not to clamp -- against plain integer
sums: every length 1..260, both start parities of each stream, random data.
Built with AddressSanitizer, each stream in a heap block that ends at its
last sample, so a read past any stream fails the test."""
import os
import subprocess

from conftest import ROOT


def test_exact_correlators_match_plain_sums(tmp_path):
    exe = str(tmp_path / "xcorr_check")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address", "-fno-omit-frame-pointer",
                    "-I" + os.path.join(ROOT, "pairphone_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "xcorr_check.cpp"), "-o", exe],
                   check=True)
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "OK 0 mismatches" in out.stdout
