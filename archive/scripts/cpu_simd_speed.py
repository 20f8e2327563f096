"""Single-thread speed of the library CPU path (sd_cpu_checksums of one 512 MiB range) at the
SIMD width SD_CPU_LANES selects: SD_CPU_LANES=8 python scripts/cpu_simd_speed.py"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, time, sys
from spacedrive_amd._native import lib, check
from spacedrive_amd import cpu
n=1<<29
d=np.random.default_rng(0).integers(0,256,n,dtype=np.uint8)
offs=np.zeros(1,np.uint64); lens=np.array([n],np.uint64); out=np.zeros(32,np.uint8)
best=1e9
for _ in range(3):
    t0=time.perf_counter(); check(lib().sd_cpu_checksums(d.ctypes.data, offs.ctypes.data, lens.ctypes.data, 1, out.ctypes.data, 1)); best=min(best,time.perf_counter()-t0)
print(cpu.simd_lanes(), "lanes 1 thread", round(n/best/1e9,3), "GB/s", out[:4])
