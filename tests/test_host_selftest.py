"""The GPU-free host core's own selftest (spacedrive_amd/csrc/host_selftest.cpp: planners,
stager, readers, pools, host thread budget, CPU path, coalescer, exchange plan, shared-range
pick, NUMA placement), built with g++ from the library's host sources and run as a child
process.  The same binary runs under ASan+UBSan and TSan with `make sanitize`
(profiles/r4/sanitize_*.txt)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "spacedrive_amd", "csrc")


def test_host_selftest():
    b = subprocess.run(["make", "-C", CSRC, "-j8", "selftest"], capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stdout[-2000:] + b.stderr[-2000:]
    r = subprocess.run([os.path.join(ROOT, "build", "csrc", "plain", "selftest")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "host_selftest: ok" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
