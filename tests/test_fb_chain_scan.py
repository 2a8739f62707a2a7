"""The exactness argument of fb_chain_scan (lmm_fb_kernels.hpp), checked on the CPU (the 64-lane fb_chain_scan and the 256-thread fb_long_chain, whose int64 prefix wraps on
steps of out-of-binade sentinels).

fbk_update_seq must reproduce the reference's element-by-element `double_update` chain bit for bit
(fair_bottleneck.cpp:110-116).  The device chains non-negative batches wave-parallel: within one binade the
rounded chain is an integer prefix sum in units of the binade's ulp, and only the steps that leave the binade
or are exact ties are taken as fp64 subtractions.  tests/c/chain_scan_check.cpp runs that algorithm (lanes
emulated, same integer arithmetic) against the sequential loop on batches built to hit ties, binade
crossings, exact landings on powers of two and values falling below the precision; the device path itself is
pinned by the bit-identical C5 tests (tests/test_gpu_configs.py).
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_chain_scan_matches_sequential_chain(tmp_path):
    exe = tmp_path / "chain_scan_check"
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-o", str(exe),
                           os.path.join(ROOT, "tests", "c", "chain_scan_check.cpp")])
    out = subprocess.run([str(exe), "40000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok 40000 batches"), out.stdout
