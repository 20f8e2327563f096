"""Generates scripts/valu_probe7.hip: per-op and per-mix VALU issue rates on gfx950, and
the BLAKE3 G function written several ways, in one harness that fits 8 waves per SIMD
(hard-named VGPRs v8..v47 only, so <= 64 VGPRs are allocated).

Each kind is an asm block of independent instruction streams; the kernel repeats it.
Readings per kind: wall-clock lane-ops/s (HIP events over 5 launches), and from the
waves' own s_memtime spans the cycles per wave-instruction per SIMD (2.0 = the SIMD-32
full rate of MI355X_MICROARCH.md; 4.0 = half rate).
python scripts/gen_valu_probe7.py  (writes the .hip; build line in its header)"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))

# registers: d = v8..v15 (dst), a = v16..v23, b = v24..v31, c = v32..v39, spare v40..v47
D = [f"v{8 + i}" for i in range(8)]
A = [f"v{16 + i}" for i in range(8)]
Bv = [f"v{24 + i}" for i in range(8)]
C = [f"v{32 + i}" for i in range(8)]


def x8(fmt):
    return [fmt.format(d=D[i], a=A[i], b=Bv[i], c=C[i]) for i in range(8)]


SINGLE = [
    ("v_xor_b32", "v_xor_b32 {d}, {a}, {b}"),
    ("v_add_u32", "v_add_u32 {d}, {a}, {b}"),
    ("v_sub_u32", "v_sub_u32 {d}, {a}, {b}"),
    ("v_or_b32", "v_or_b32 {d}, {a}, {b}"),
    ("v_and_b32", "v_and_b32 {d}, {a}, {b}"),
    ("v_lshrrev_b32 (const)", "v_lshrrev_b32 {d}, 7, {a}"),
    ("v_lshlrev_b32 (const)", "v_lshlrev_b32 {d}, 25, {a}"),
    ("v_lshrrev_b32 (vgpr)", "v_lshrrev_b32 {d}, {b}, {a}"),
    ("v_cndmask_b32", "v_cndmask_b32 {d}, {a}, {b}, vcc"),
    ("v_mov_b32", "v_mov_b32 {d}, {a}"),
    ("v_add_co_u32 (VOP2, carry out)", "v_add_co_u32 {d}, vcc, {a}, {b}"),
    ("v_fma_f32", "v_fma_f32 {d}, {a}, {b}, {c}"),
    ("v_bitop3_b32", "v_bitop3_b32 {d}, {a}, {b}, {c} bitop3:0x96"),
    ("v_bfi_b32", "v_bfi_b32 {d}, {a}, {b}, {c}"),
    ("v_add3_u32", "v_add3_u32 {d}, {a}, {b}, {c}"),
    ("v_xad_u32", "v_xad_u32 {d}, {a}, {b}, {c}"),
    ("v_or3_b32", "v_or3_b32 {d}, {a}, {b}, {c}"),
    ("v_alignbit_b32 x,x,7", "v_alignbit_b32 {d}, {a}, {a}, 7"),
    ("v_alignbyte_b32 x,x,1", "v_alignbyte_b32 {d}, {a}, {a}, 1"),
    ("v_perm_b32", "v_perm_b32 {d}, {a}, {a}, {b}"),
    ("v_lshl_or_b32", "v_lshl_or_b32 {d}, {a}, 7, {b}"),
    ("v_lshl_add_u32", "v_lshl_add_u32 {d}, {a}, 7, {b}"),
    ("v_add_lshl_u32", "v_add_lshl_u32 {d}, {a}, {b}, {c}"),
    ("v_xor_b32_e64 (VOP3 2-src)", "v_xor_b32_e64 {d}, {a}, {b}"),
    ("v_add_u32_e64 (VOP3 2-src)", "v_add_u32_e64 {d}, {a}, {b}"),
    ("v_xor_b32_sdwa WORD_1 preserve", "v_xor_b32_sdwa {d}, {a}, {b} dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE "
                                       "src0_sel:WORD_0 src1_sel:WORD_0"),
    ("v_xor_b32 dpp row_shr:1", "v_xor_b32_dpp {d}, {a}, {b} row_shr:1 row_mask:0xf bank_mask:0xf"),
    ("v_pk_add_u16", "v_pk_add_u16 {d}, {a}, {b}"),
    ("v_mul_u32_u24", "v_mul_u32_u24 {d}, {a}, {b}"),
]


def mix(*fmts):
    """8 instructions alternating the given forms (independent registers)."""
    return [fmts[i % len(fmts)].format(d=D[i], a=A[i], b=Bv[i], c=C[i]) for i in range(8)]


MIXES = [
    ("mix xor : add3  1:1", mix("v_xor_b32 {d}, {a}, {b}", "v_add3_u32 {d}, {a}, {b}, {c}")),
    ("mix xor : alignbit 1:1", mix("v_xor_b32 {d}, {a}, {b}", "v_alignbit_b32 {d}, {a}, {a}, 7")),
    ("mix fma_f32 : add3 1:1", mix("v_fma_f32 {d}, {a}, {b}, {c}", "v_add3_u32 {d}, {a}, {b}, {c}")),
    ("mix bitop3 : alignbit 1:1", mix("v_bitop3_b32 {d}, {a}, {b}, {c} bitop3:0x96", "v_alignbit_b32 {d}, {a}, {a}, 7")),
    ("mix xor x3 : add3 x1", mix("v_xor_b32 {d}, {a}, {b}", "v_xor_b32 {d}, {a}, {b}", "v_xor_b32 {d}, {a}, {b}",
                                 "v_add3_u32 {d}, {a}, {b}, {c}")),
    ("mix xor x1 : add3 x3", mix("v_xor_b32 {d}, {a}, {b}", "v_add3_u32 {d}, {a}, {b}, {c}",
                                 "v_add3_u32 {d}, {a}, {b}, {c}", "v_add3_u32 {d}, {a}, {b}, {c}")),
]


# --- the G function, 4 independent columns, one round (48 or more instructions) --------
# column k: a = v(8+k), b = v(12+k), c = v(16+k), d = v(20+k), m0 = v(24+k), m1 = v(28+k),
#           t = v(32+k), u = v(36+k)
def g_variant(kind):
    out = []
    cols = range(4)

    def r(name, k):
        base = {"a": 8, "b": 12, "c": 16, "d": 20, "m0": 24, "m1": 28, "t": 32, "u": 36}[name]
        return f"v{base + k}"

    def emit(fmt):  # one op per column, interleaved op by op (4 independent chains)
        for k in cols:
            out.append(fmt.format(**{n: r(n, k) for n in ("a", "b", "c", "d", "m0", "m1", "t", "u")}))

    def rot(dst, src, n):
        if kind == "shift_or":
            emit(f"v_lshrrev_b32 {{u}}, {n}, {src}")
            emit(f"v_lshlrev_b32 {dst}, {32 - n}, {src}")
            emit(f"v_or_b32 {dst}, {dst}, {{u}}")
        else:
            emit(f"v_alignbit_b32 {dst}, {src}, {src}, {n}")

    def add3(dst, x, y, z):
        if kind == "split_add3":
            emit(f"v_add_u32 {dst}, {x}, {y}")
            emit(f"v_add_u32 {dst}, {dst}, {z}")
        else:
            emit(f"v_add3_u32 {dst}, {x}, {y}, {z}")

    add3("{a}", "{a}", "{b}", "{m0}")
    if kind in ("sdwa16", "split_add3"):  # rotr(d ^ a, 16) as two crosswise SDWA xors
        emit("v_xor_b32_sdwa {t}, {d}, {a} dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1")
        emit("v_xor_b32_sdwa {t}, {d}, {a} dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0")
    elif kind == "perm16":
        emit("v_xor_b32 {t}, {d}, {a}")
        emit("v_perm_b32 {t}, {t}, {t}, s4")
    else:
        emit("v_xor_b32 {t}, {d}, {a}")
        rot("{t}", "{t}", 16)
    emit("v_add_u32 {c}, {c}, {t}")
    emit("v_xor_b32 {b}, {b}, {c}")
    rot("{b}", "{b}", 12)
    add3("{a}", "{a}", "{b}", "{m1}")
    emit("v_xor_b32 {d}, {t}, {a}")
    rot("{d}", "{d}", 8)
    emit("v_add_u32 {c}, {c}, {d}")
    emit("v_xor_b32 {b}, {b}, {c}")
    rot("{b}", "{b}", 7)
    return out


GS = [
    ("G: add3 + sdwa16 + alignbit (the kernels' G)", g_variant("sdwa16")),
    ("G: add3 + alignbit x4", g_variant("alignbit")),
    ("G: add3 + perm16 + alignbit", g_variant("perm16")),
    ("G: add3 split in 2 adds + sdwa16", g_variant("split_add3")),
    ("G: add3 + rotates as shift/shift/or", g_variant("shift_or")),
]


def asm_str(lines):
    return "".join(f'"{ln}\\n"' for ln in lines)


def main():
    kinds = [(n, x8(f)) for n, f in SINGLE] + MIXES + GS
    body = []
    for k, (name, lines) in enumerate(kinds):
        body.append(f"    if (KIND == {k}) asm volatile({asm_str(lines)} ::: CLOB);")
    names = ",\n    ".join(f'{{"{n}", {len(l)}}}' for n, l in kinds)
    src = f'''// GENERATED by scripts/gen_valu_probe7.py -- VALU issue rates per op, per mix and per way
// of writing BLAKE3's G, on gfx950, at 1/2/4/8 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -w -o scripts/valu_probe7 scripts/valu_probe7.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define REP 8
#define CLOB "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", \\
    "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36",  \\
    "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "vcc", "s4"
struct Kind {{
    const char* name;
    int instrs;  // per asm block
}};
static const Kind kKinds[] = {{
    {names}}};
constexpr int NKINDS = {len(kinds)};

template <int KIND>
__global__ __launch_bounds__(256) void k_op(uint64_t* cyc, uint32_t iters) {{
    asm volatile(
        "v_mov_b32 v8, 1\\nv_mov_b32 v9, 2\\nv_mov_b32 v10, 3\\nv_mov_b32 v11, 4\\nv_mov_b32 v12, 5\\n"
        "v_mov_b32 v13, 6\\nv_mov_b32 v14, 7\\nv_mov_b32 v15, 8\\nv_mov_b32 v16, 9\\nv_mov_b32 v17, 10\\n"
        "v_mov_b32 v18, 11\\nv_mov_b32 v19, 12\\nv_mov_b32 v20, 13\\nv_mov_b32 v21, 14\\nv_mov_b32 v22, 15\\n"
        "v_mov_b32 v23, 16\\nv_mov_b32 v24, 17\\nv_mov_b32 v25, 18\\nv_mov_b32 v26, 19\\nv_mov_b32 v27, 20\\n"
        "v_mov_b32 v28, 21\\nv_mov_b32 v29, 22\\nv_mov_b32 v30, 23\\nv_mov_b32 v31, 24\\nv_mov_b32 v32, 25\\n"
        "v_mov_b32 v33, 26\\nv_mov_b32 v34, 27\\nv_mov_b32 v35, 28\\nv_mov_b32 v36, 29\\nv_mov_b32 v37, 30\\n"
        "v_mov_b32 v38, 31\\nv_mov_b32 v39, 32\\nv_mov_b32 v40, 33\\nv_mov_b32 v41, 34\\nv_mov_b32 v42, 35\\n"
        "v_mov_b32 v43, 36\\nv_mov_b32 v44, 37\\nv_mov_b32 v45, 38\\nv_mov_b32 v46, 39\\nv_mov_b32 v47, 40\\n"
        "s_mov_b64 vcc, 0\\ns_mov_b32 s4, 0x01000302" ::: CLOB);
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t it = 0; it < iters; it++) {{
#pragma unroll
        for (int r = 0; r < REP; r++) {{
{chr(10).join(body)}
        }}
    }}
    __syncthreads();
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t v;
    asm volatile("v_mov_b32 %0, v8" : "=v"(v));
    if (threadIdx.x == 0) {{  // per-lane (vector) stores of the block's span
        cyc[2 * blockIdx.x] = t1 - t0;
        cyc[2 * blockIdx.x + 1] = (r1 - r0) + (v == 0x12345678u ? 1 : 0);
    }}
}}

template <int K>
struct Table {{
    static void fill(void (**f)(uint64_t*, uint32_t)) {{
        f[K] = k_op<K>;
        Table<K + 1>::fill(f);
    }}
}};
template <>
struct Table<NKINDS> {{
    static void fill(void (**)(uint64_t*, uint32_t)) {{}}
}};

int main() {{
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    void (*fns[NKINDS])(uint64_t*, uint32_t);
    Table<0>::fill(fns);
    const int cus = p.multiProcessorCount;
    hipFuncAttributes fa;
    (void)hipFuncGetAttributes(&fa, (const void*)fns[0]);
    printf("# %s, %d CUs, %d VGPRs/lane in the probe kernel; wall = HIP events over 5 launches; cyc = median "
           "workgroup s_memtime span / (waves per SIMD x instructions per wave)\\n",
           p.gcnArchName, cus, fa.numRegs);
    printf("# %-3s %-48s %9s %12s %8s %6s\\n", "wps", "kind", "T lane/s", "lane/clk/CU", "cyc/ins", "MHz");
    for (int wps : {{1, 2, 4, 8}}) {{
        const int grid = cus * wps;
        uint64_t* cyc;
        (void)hipMalloc(&cyc, (size_t)grid * 16);
        for (int k = 0; k < NKINDS; k++) {{
            const uint32_t iters = (uint32_t)(4096 * 8 / kKinds[k].instrs);  // ~32k instructions per block pass
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            for (int w = 0; w < 10; w++) hipLaunchKernelGGL(fns[k], dim3(grid), dim3(256), 0, 0, cyc, iters);
            (void)hipEventRecord(e0);
            for (int r = 0; r < 5; r++) hipLaunchKernelGGL(fns[k], dim3(grid), dim3(256), 0, 0, cyc, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            std::vector<uint64_t> h((size_t)grid * 2);
            (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
            std::vector<double> c(grid), mhz(grid);
            for (int b = 0; b < grid; b++) {{
                c[b] = (double)h[2 * b];
                mhz[b] = (double)h[2 * b] / ((double)h[2 * b + 1] / 100.0);  // s_memrealtime: 100 MHz
            }}
            std::sort(c.begin(), c.end());
            std::sort(mhz.begin(), mhz.end());
            const double per_wave = (double)iters * REP * kKinds[k].instrs;
            const double ops = 5.0 * grid * 256.0 * per_wave;
            printf("  %-3d %-48s %9.2f %12.1f %8.2f %6.0f\\n", wps, kKinds[k].name, ops / (ms * 1e-3) / 1e12,
                   per_wave * 64.0 * 4 * wps / c[grid / 2], c[grid / 2] / (wps * per_wave), mhz[grid / 2]);
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
        }}
        (void)hipFree(cyc);
    }}
    return 0;
}}
'''
    open(os.path.join(HERE, "valu_probe7.hip"), "w").write(src)


if __name__ == "__main__":
    main()
