"""Generates scripts/valu_probe8.hip: does gfx950's FP64 VALU issue beside the half-rate
integer ops, the way probe7 found fp32 FMA does (`mix fma_f32 : add3 1:1` at 67.8 T)?

Why: a 64-bit register pair whose high word is small is a denormal double whose bit
pattern IS the integer, and v_add_f64 of two such patterns is exact integer addition up
to 2^53 -- so the low word of the sum is the 32-bit modular add BLAKE3 needs, and the
carry lands in the high word, which nothing reads.  If FP64 adds overlap the integer
pipe, BLAKE3's six adds per G can leave it.

Each kind is an asm block; the kernel repeats it.  Registers v8..v63 only (8 waves/SIMD
fit); even registers start at small integers and odd ones at 0, so every pair is a small
denormal.
python scripts/gen_valu_probe8.py  (writes the .hip; build line in its header)"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def P(r):  # register pair starting at an even register
    return f"v[{r}:{r + 1}]"


# pure streams: 8 independent instructions, dst pairs v8..v23, sources v24..v55
def f64x8(op, n_src=2):
    out = []
    for i in range(8):
        d = 8 + 2 * i
        a, b, c = 24 + 2 * (i % 4), 32 + 2 * (i % 4), 40 + 2 * (i % 4)
        srcs = [P(a), P(b), P(c)][:n_src]
        out.append(f"{op} {P(d)}, " + ", ".join(srcs))
    return out


def i32x8(fmt):
    return [fmt.format(d=f"v{8 + i}", a=f"v{24 + i}", b=f"v{32 + i}", c=f"v{40 + i}") for i in range(8)]


ADD3 = "v_add3_u32 {d}, {a}, {b}, {c}"
ALIGN = "v_alignbit_b32 {d}, {a}, {a}, 7"
XOR = "v_xor_b32 {d}, {a}, {b}"


def mix_f64_int(f64op, int_fmts, pattern):
    """pattern: string of 'f' (an f64 op) and 'i' (the next int op); independent registers.
    f64 ops write pairs v8..v23 (round-robin); int ops write v56..v63."""
    out, fi, ii = [], 0, 0
    for ch in pattern:
        if ch == "f":
            d = 8 + 2 * (fi % 8)
            out.append(f"{f64op} {P(d)}, {P(24 + 2 * (fi % 4))}, {P(32 + 2 * (fi % 4))}")
            fi += 1
        else:
            fmt = int_fmts[ii % len(int_fmts)]
            out.append(fmt.format(d=f"v{56 + ii % 8}", a=f"v{41 + ii % 8}", b=f"v{49 + ii % 7}",
                                  c=f"v{25 + 2 * (ii % 4)}"))
            ii += 1
    return out


SINGLE = [
    ("v_xor_b32 (control)", i32x8(XOR)),
    ("v_add3_u32 (control)", i32x8(ADD3)),
    ("v_alignbit_b32 (control)", i32x8(ALIGN)),
    ("v_fma_f32 (control)", i32x8("v_fma_f32 {d}, {a}, {b}, {c}")),
    ("v_add_f64 (denormal pairs)", f64x8("v_add_f64")),
    ("v_mul_f64", f64x8("v_mul_f64")),
    ("v_fma_f64", f64x8("v_fma_f64", 3)),
    ("v_pk_add_f32", f64x8("v_pk_add_f32")),
    ("v_pk_fma_f32", f64x8("v_pk_fma_f32", 3)),
    ("v_pk_mov_b32", [f"v_pk_mov_b32 {P(8 + 2 * i)}, {P(24 + 2 * (i % 4))}, {P(32 + 2 * (i % 4))} op_sel:[0,1]"
                      for i in range(8)]),
    ("v_lshlrev_b64", [f"v_lshlrev_b64 {P(8 + 2 * i)}, 7, {P(24 + 2 * (i % 4))}" for i in range(8)]),
    ("v_lshrrev_b64", [f"v_lshrrev_b64 {P(8 + 2 * i)}, 7, {P(24 + 2 * (i % 4))}" for i in range(8)]),
]

MIXES = [
    ("mix add_f64 : add3 1:1", mix_f64_int("v_add_f64", [ADD3], "fifififi")),
    ("mix add_f64 : alignbit 1:1", mix_f64_int("v_add_f64", [ALIGN], "fifififi")),
    ("mix add_f64 : xor 1:1", mix_f64_int("v_add_f64", [XOR], "fifififi")),
    ("mix add_f64 x1 : (xor,alignbit) x2", mix_f64_int("v_add_f64", [XOR, ALIGN], "fiifiifiifii")),
    ("mix add_f64 x1 : (add3,alignbit) x2", mix_f64_int("v_add_f64", [ADD3, ALIGN], "fiifiifiifii")),
    ("mix add_f64 x3 : alignbit x4", mix_f64_int("v_add_f64", [ALIGN], "fififif" + "i" * 1 + "fififif" + "i")),
    ("mix mul_f64 : alignbit 1:1", mix_f64_int("v_mul_f64", [ALIGN], "fifififi")),
    ("mix pk_add_f32 : alignbit 1:1", mix_f64_int("v_pk_add_f32", [ALIGN], "fifififi")),
    ("mix pk_add_f32 : xor 1:1", mix_f64_int("v_pk_add_f32", [XOR], "fifififi")),
]


# --- the G function, 4 independent columns, one round -------------------------------------
# column k: pairs a = v(8+2k), b = v(16+2k), c = v(24+2k), d = v(32+2k), t = v(40+2k),
#           m0 = v(48+2k), m1 = v(56+2k); the low word of a pair is its even register.
def g_variant(kind):
    out = []

    def r(name, k, hi=False):
        base = {"a": 8, "b": 16, "c": 24, "d": 32, "t": 40, "m0": 48, "m1": 56}[name]
        return f"v{base + 2 * k + (1 if hi else 0)}"

    def emit(fmt):
        for k in range(4):
            kw = {n: r(n, k) for n in ("a", "b", "c", "d", "t", "m0", "m1")}
            kw.update({n.upper(): P(int(r(n, k)[1:])) for n in ("a", "b", "c", "d", "t", "m0", "m1")})
            kw.update({n + "h": r(n, k, True) for n in ("a", "b", "c", "d", "t")})
            out.append(fmt.format(**kw))

    int_add = kind == "int"
    m_f64 = kind in ("f64_all", "f64_all_rot12")

    def add_abm(m):
        if int_add:
            emit(f"v_add3_u32 {{a}}, {{a}}, {{b}}, {{{m}}}")
        elif m_f64:
            emit(f"v_add_f64 {{A}}, {{A}}, {{{m.upper()}}}")
            emit("v_add_f64 {A}, {A}, {B}")
        else:
            emit(f"v_add_u32 {{a}}, {{a}}, {{{m}}}")
            emit("v_add_f64 {A}, {A}, {B}")

    def add_cd(dn):
        if int_add:
            emit(f"v_add_u32 {{c}}, {{c}}, {{{dn}}}")
        else:
            emit(f"v_add_f64 {{C}}, {{C}}, {{{dn.upper()}}}")

    add_abm("m0")
    emit("v_xor_b32_sdwa {t}, {d}, {a} dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1")
    emit("v_xor_b32_sdwa {t}, {d}, {a} dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0")
    add_cd("t")
    emit("v_xor_b32 {b}, {b}, {c}")
    if kind == "f64_all_rot12":  # rotr(x,12): pattern x * 2^20 (exact below 2^53), low | high
        emit("v_mul_f64 {D}, {B}, s[6:7]")  # d is dead here (rewritten below); s[6:7] = 2^20 as a double
        emit("v_or_b32 {b}, {d}, {dh}")
    else:
        emit("v_alignbit_b32 {b}, {b}, {b}, 12")
    add_abm("m1")
    emit("v_xor_b32 {d}, {t}, {a}")
    emit("v_alignbit_b32 {d}, {d}, {d}, 8")
    add_cd("d")
    emit("v_xor_b32 {b}, {b}, {c}")
    emit("v_alignbit_b32 {b}, {b}, {b}, 7")
    return out


GS = [
    ("G: the kernels' G (int)", g_variant("int")),
    ("G: a+=b, c+=d in f64 (m by v_add_u32)", g_variant("f64_ab_cd")),
    ("G: all 6 adds in f64", g_variant("f64_all")),
    ("G: all 6 adds in f64 + rotr12 by mul_f64", g_variant("f64_all_rot12")),
]


def asm_str(lines):
    return "".join(f'"{ln}\\n"' for ln in lines)


def main():
    kinds = SINGLE + MIXES + GS
    body = []
    for k, (name, lines) in enumerate(kinds):
        body.append(f"    if (KIND == {k}) asm volatile({asm_str(lines)} ::: CLOB);")
    names = ",\n    ".join(f'{{"{n}", {len(l)}, {sum(1 for x in l if "_f64" in x or "_f32" in x)}}}'
                           for n, l in kinds)
    init = "".join(f'"v_mov_b32 v{r}, {(r // 2) if r % 2 == 0 else 0}\\n"' for r in range(8, 64))
    clob = ", ".join(f'"v{r}"' for r in range(8, 64))
    src = f'''// GENERATED by scripts/gen_valu_probe8.py -- FP64 / packed-FP32 VALU issue beside the
// half-rate integer ops on gfx950, and BLAKE3's G with its adds as f64 adds of denormal
// register pairs.  Build: hipcc --offload-arch=gfx950 -O3 -w -o scripts/valu_probe8 scripts/valu_probe8.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define REP 8
#define CLOB {clob}, "vcc", "s4", "s6", "s7"
struct Kind {{
    const char* name;
    int instrs;  // per asm block
    int fp;      // of which fp (f64 or packed f32) instructions
}};
static const Kind kKinds[] = {{
    {names}}};
constexpr int NKINDS = {len(kinds)};

template <int KIND>
__global__ __launch_bounds__(256) void k_op(uint64_t* cyc, uint32_t iters) {{
    asm volatile({init}
        "s_mov_b64 vcc, 0\\ns_mov_b32 s4, 0x01000302\\ns_mov_b32 s6, 0\\ns_mov_b32 s7, 0x41300000" ::: CLOB);
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
    printf("# %s, %d CUs, %d VGPRs/lane in the probe kernel; wall = HIP events over 5 launches\\n", p.gcnArchName,
           cus, fa.numRegs);
    printf("# %-3s %-44s %9s %11s %8s %6s\\n", "wps", "kind", "T ins/s", "ins/clk/CU", "G/ns/CU", "MHz");
    for (int wps : {{4, 8}}) {{
        const int grid = cus * wps;
        uint64_t* cyc;
        (void)hipMalloc(&cyc, (size_t)grid * 16);
        for (int k = 0; k < NKINDS; k++) {{
            const uint32_t iters = (uint32_t)(4096 * 8 / kKinds[k].instrs);
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
            std::vector<double> mhz(grid);
            for (int b = 0; b < grid; b++) mhz[b] = (double)h[2 * b] / ((double)h[2 * b + 1] / 100.0);
            std::sort(mhz.begin(), mhz.end());
            const double per_wave = (double)iters * REP * kKinds[k].instrs;
            const double ops = 5.0 * grid * 256.0 * per_wave;  // lane-instructions
            const double tps = ops / (ms * 1e-3);
            const double clk = mhz[grid / 2] * 1e6;
            // G/ns/CU: for the G kinds, G functions (4 per block) per ns per CU
            const double gs = (double)iters * REP * 4 * 5.0 * grid * 256.0 / (ms * 1e-3) / 1e9 / cus;
            printf("  %-3d %-44s %9.2f %11.1f %8.3f %6.0f\\n", wps, kKinds[k].name, tps / 1e12,
                   tps / (cus * clk), gs, mhz[grid / 2]);
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
        }}
        (void)hipFree(cyc);
    }}
    return 0;
}}
'''
    open(os.path.join(HERE, "valu_probe8.hip"), "w").write(src)


if __name__ == "__main__":
    main()
