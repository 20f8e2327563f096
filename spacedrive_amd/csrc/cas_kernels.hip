// cas_kernels.hip -- gfx950 kernels for Spacedrive's content-addressing hot path.
//
//   k_cas_sampled_lanes  generate_cas_id, size > 102400 (cas.rs:30-58): every message is
//   k_cas_sampled_merge  the same 57 352 B = 56 full chunks + one 8-byte chunk, so one lane
//                   per aligned 8-chunk group (7 per file) hashes its subtree, and one lane
//                   per file merges the 7 subtree CVs and the tail chunk.  No work lists.
//   k_whole_items   generate_cas_id, size <= 102400 (cas.rs:27-29): host-built work lists
//   k_whole_merge8  of aligned chunk pairs (full pairs of multi-pair messages, then the
//                   cost-sorted partial / short pairs), then two level-wise merge passes of
//                   <= 8 pair nodes per lane.
//   k_ck_leaf       file_checksum (hash.rs:10-24), and whole-file cas messages longer than
//   k_ck_reduce     the work-list path takes: 256 lanes per 1 MiB block of a message, two
//                   blocks per workgroup, 4 consecutive chunks per lane merged in-lane, each
//                   block's 256 lane CVs merged in LDS (both trees packed into the lowest
//                   lanes); then 256-way LDS reductions over the block CVs.
//
// Tree shape: every merge is the level-wise pairwise merge with the odd node carried up
// unchanged, over power-of-two aligned groups.  It is the BLAKE3 tree (left subtree =
// largest power of two); tests/test_oracle.py checks the equivalence for 1..600 chunks.
#include <hip/hip_runtime.h>

#include "blake3_device.h"
#include "sd_internal.h"

using namespace sdb3;

namespace {

__device__ __forceinline__ void store_cv(uint32_t* dst, const uint32_t (&cv)[8]) {
    uint4* d = reinterpret_cast<uint4*>(dst);
    d[0] = make_uint4(cv[0], cv[1], cv[2], cv[3]);
    d[1] = make_uint4(cv[4], cv[5], cv[6], cv[7]);
}
__device__ __forceinline__ void load_cv(uint32_t (&cv)[8], const uint32_t* src) {
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4 a = s[0], b = s[1];
    cv[0] = a.x; cv[1] = a.y; cv[2] = a.z; cv[3] = a.w;
    cv[4] = b.x; cv[5] = b.y; cv[6] = b.z; cv[7] = b.w;
}

// Level-wise merge of n (1..blockDim) CVs held in lds[0..n) -> lds[0].  ROOT goes on the
// final parent when `root`.  Every thread of the workgroup must call it.
__device__ void lds_reduce(uint32_t (*lds)[8], uint32_t n, bool root) {
    const uint32_t t = threadIdx.x;
    while (n > 1) {
        const uint32_t P = n >> 1;
        const bool carry = n & 1u;
        uint32_t res[8];
        bool have = false;
        if (t < P) {
            uint32_t l[8], r[8];
            load_cv(l, lds[2 * t]);
            load_cv(r, lds[2 * t + 1]);
            parent(res, l, r, (root && n == 2) ? ROOT : 0u);
            have = true;
        } else if (carry && t == P) {
            load_cv(res, lds[n - 1]);
            have = true;
        }
        __syncthreads();
        if (have) store_cv(lds[t], res);
        __syncthreads();
        n = P + (carry ? 1u : 0u);
    }
}

}  // namespace

// ------------------------------------------------------------------------ sampled cas
// Every sampled message is the same 57 352 B = 56 full chunks + one 8-byte chunk (message
// bytes 57344..57351, chunk 56), so the launch shape needs no work lists:
constexpr int S_FULL = 56;  // full chunks per sampled message (57344 bytes)
#ifndef SD_SAMPLED_LANE_CHUNKS
#define SD_SAMPLED_LANE_CHUNKS 8  // chunks per lane (2, 4 or 8; scripts/sampled_ab.py)
#endif
constexpr int S_U = SD_SAMPLED_LANE_CHUNKS;
constexpr int S_K = S_FULL / S_U;  // nodes per file after the lanes kernel (7)
static_assert(S_U == 2 || S_U == 4 || S_U == 8, "chunks per lane");

// Two kernels, and no in-workgroup tree phase (round 2 measured a one-kernel design -- 16
// files per 7-wave workgroup, the 29 lane CVs of each merged level-wise in LDS -- 3.4%
// slower: the LDS rounds, barriers and partly-filled waves of its tree phase cost more than
// a second launch; profiles/r2/r2z_sampled_ab.json):
//   k_cas_sampled_lanes<U>  one lane per (file, aligned group of U chunks): 56/U lanes per
//                           file, 256-lane workgroups, no LDS, no barrier; the group's
//                           subtree CV -> node row j of the file, rows stored node-major
//                           (row (j, f) at (j * n + f) * 32 B) so the merge reads coalesce;
//   k_cas_sampled_merge<U>  one lane per file: the 56/U node CVs merged with BLAKE3's CV
//                           stack, then the 8-byte tail chunk (chunk 56) and the stack folded
//                           into the root.
// CvStack: the pending subtree CVs, top first, in registers with static indices only (a
// push shifts every entry down one slot), so a loop that is not unrolled can drive it.
template <int D>
struct CvStack {
    uint32_t s[D][8];
    __device__ __forceinline__ void push(const uint32_t (&c)[8]) {
#pragma unroll
        for (int d = D - 1; d > 0; d--)
#pragma unroll
            for (int i = 0; i < 8; i++) s[d][i] = s[d - 1][i];
#pragma unroll
        for (int i = 0; i < 8; i++) s[0][i] = c[i];
    }
    // c <- parent(top, c), and the top popped
    __device__ __forceinline__ void merge_top(uint32_t (&c)[8], uint32_t flags) {
        uint32_t r[8];
        parent(r, s[0], c, flags);
#pragma unroll
        for (int i = 0; i < 8; i++) c[i] = r[i];
#pragma unroll
        for (int d = 0; d + 1 < D; d++)
#pragma unroll
            for (int i = 0; i < 8; i++) s[d][i] = s[d + 1][i];
    }
};

constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x / 2); }

// CV of U (a power of two) consecutive full non-root chunks c0.. : U = 2 is full_chunks_cv's
// unrolled pair; larger groups merge each chunk into the stack as it completes.
template <int U>
__device__ __forceinline__ void group_cv(uint32_t (&out)[8], const uint8_t* __restrict__ p, uint64_t c0) {
    if constexpr (U <= 2) {
        full_chunks_cv<U>(out, p, c0);
    } else {
        CvStack<ilog2(U)> st;
        uint32_t ma[16], mb[16];
#pragma unroll 1
        for (uint32_t u = 0; u < (uint32_t)U; u++) {
            const uint64_t ctr = c0 + u;
            const uint32_t clo = (uint32_t)ctr, chi = (uint32_t)(ctr >> 32);
            const uint8_t* q = p + (size_t)u * CHUNK_LEN;
            set_iv(out);
#pragma unroll 1
            for (uint32_t b = 0; b < 16; b += 2) {
                load_block(ma, q + 64u * b);
                load_block(mb, q + 64u * (b + 1));
                compress(out, ma, clo, chi, BLOCK_LEN, b == 0 ? CHUNK_START : 0u);
                compress(out, mb, clo, chi, BLOCK_LEN, b + 1 == 15 ? CHUNK_END : 0u);
            }
#pragma unroll 1
            for (uint32_t t = u + 1; (t & 1u) == 0; t >>= 1) st.merge_top(out, 0u);
            if (u + 1 < (uint32_t)U) st.push(out);
        }
    }
}

template <int U>
__global__ __launch_bounds__(256) void k_cas_sampled_lanes(const uint8_t* __restrict__ staged,
                                                           const uint64_t* __restrict__ soff, uint32_t n,
                                                           uint32_t* __restrict__ rows) {
    constexpr uint32_t K = S_FULL / U;
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (uint64_t)n * K) return;
    const uint32_t f = (uint32_t)(g / K), j = (uint32_t)(g - (uint64_t)f * K);
    uint32_t cv[8];
    group_cv<U>(cv, staged + soff[f] + (size_t)j * U * CHUNK_LEN, (uint64_t)j * U);
    store_cv(rows + ((size_t)j * n + f) * 8, cv);
}

template <int U>
__global__ __launch_bounds__(256) void k_cas_sampled_merge(const uint8_t* __restrict__ staged,
                                                           const uint64_t* __restrict__ soff,
                                                           const uint32_t* __restrict__ idx, uint32_t n,
                                                           const uint32_t* __restrict__ rows, uint32_t* __restrict__ out) {
    constexpr uint32_t K = S_FULL / U;
    constexpr int D = ilog2(K + 1);  // after node k the stack holds popcount(k + 1) subtrees
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n) return;
    CvStack<D> st;
    uint32_t cur[8], nxt[8];
    load_cv(nxt, rows + (size_t)f * 8);
#pragma unroll 1
    for (uint32_t k = 0; k < K; k++) {
#pragma unroll
        for (int i = 0; i < 8; i++) cur[i] = nxt[i];
        if (k + 1 < K) load_cv(nxt, rows + ((size_t)(k + 1) * n + f) * 8);  // in flight during the merges
#pragma unroll 1
        for (uint32_t t = k + 1; (t & 1u) == 0; t >>= 1) st.merge_top(cur, 0u);
        st.push(cur);
    }
    // the tail chunk is the rightmost node; the stack's subtrees fold onto it, ROOT last
    chunk_cv(cur, staged + soff[f] + (size_t)S_FULL * CHUNK_LEN, SD_SAMPLED_MSG_LEN - S_FULL * CHUNK_LEN, S_FULL,
             false);
    constexpr int P = __builtin_popcount(K);  // subtrees on the stack after K nodes
#pragma unroll 1
    for (int d = 0; d < P; d++) st.merge_top(cur, d + 1 == P ? ROOT : 0u);
    store_cv(out + (size_t)idx[f] * 8, cur);
}

// Small batches (latency): the kernels above trade per-file latency for throughput -- one
// lane walks 8 chunks (135 dependent compressions) and the merge adds 8 more, fine when
// tens of thousands of files fill the chip, but a watcher event or a 100-file identifier
// step then waits for that whole chain.  k_cas_sampled_wave: one 64-lane wave per file,
// one full chunk per lane (lanes 0..55; the next line pair in flight while the current one
// is compressed), lane 56 the 8-byte tail chunk, then the 57 chunk CVs merged level-wise
// in LDS (6 levels): 16 + 6 dependent compressions per file.
// Full 1 KiB non-root chunk, the next line pair in flight while the current one is
// compressed: latency kernels (one chunk per lane, few waves) that cannot hide the load
// of each line pair behind other waves.
__device__ __forceinline__ void full_chunk_cv_prefetch(uint32_t (&cv)[8], const uint8_t* __restrict__ q,
                                                       uint32_t counter) {
    set_iv(cv);
    uint32_t ma[16], mb[16], na[16], nb[16];
    load_block(ma, q);
    load_block(mb, q + 64);
#pragma unroll
    for (uint32_t b = 0; b < 16; b += 2) {
        if (b + 2 < 16) {
            load_block(na, q + 64u * (b + 2));
            load_block(nb, q + 64u * (b + 3));
        }
        compress(cv, ma, counter, 0u, BLOCK_LEN, b == 0 ? CHUNK_START : 0u);
        compress(cv, mb, counter, 0u, BLOCK_LEN, b + 1 == 15 ? CHUNK_END : 0u);
#pragma unroll
        for (int i = 0; i < 16; i++) {
            ma[i] = na[i];
            mb[i] = nb[i];
        }
    }
}

__global__ __launch_bounds__(64) void k_cas_sampled_wave(const uint8_t* __restrict__ staged,
                                                         const uint64_t* __restrict__ soff,
                                                         const uint32_t* __restrict__ idx, uint32_t n,
                                                         uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[64][8];
    const uint32_t f = blockIdx.x, t = threadIdx.x;
    const uint8_t* msg = staged + soff[f];
    uint32_t cv[8];
    if (t < (uint32_t)S_FULL) {
        full_chunk_cv_prefetch(cv, msg + (size_t)t * CHUNK_LEN, t);
        store_cv(lds[t], cv);
    } else if (t == (uint32_t)S_FULL) {
        chunk_cv(cv, msg + (size_t)S_FULL * CHUNK_LEN, SD_SAMPLED_MSG_LEN - S_FULL * CHUNK_LEN, S_FULL, false);
        store_cv(lds[t], cv);
    }
    __syncthreads();
    lds_reduce(lds, S_FULL + 1, true);
    if (t < 8) out[(size_t)idx[f] * 8 + t] = lds[0][t];
}

// Small batches of whole-kind messages (latency; see k_cas_sampled_wave): one 128-lane
// workgroup per message of <= 101 chunks (SD_WHOLE_ITEMS_MAX), lane c hashes chunk c, the
// chunk CVs merge level-wise in LDS: at most 16 + 7 dependent compressions, against the
// work-list path's 33 (a chunk pair per lane) + two merge launches.  Row = (u64 message
// offset, message length, output row).
__global__ __launch_bounds__(128) void k_whole_wave(const uint8_t* __restrict__ staged, const uint4* __restrict__ rows,
                                                    uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[128][8];
    const uint4 r = rows[blockIdx.x];
    const uint32_t t = threadIdx.x, L = r.z;
    const uint8_t* msg = staged + ((uint64_t)r.x | ((uint64_t)r.y << 32));
    const uint32_t C = L == 0 ? 1u : (L + CHUNK_LEN - 1) / CHUNK_LEN;
    if (t < C) {
        const uint32_t len = L == 0 ? 0u : (L - t * CHUNK_LEN < CHUNK_LEN ? L - t * CHUNK_LEN : CHUNK_LEN);
        uint32_t cv[8];
        if (len == CHUNK_LEN && C > 1) full_chunk_cv_prefetch(cv, msg + (size_t)t * CHUNK_LEN, t);
        else chunk_cv(cv, msg + (size_t)t * CHUNK_LEN, len, t, C == 1);
        store_cv(lds[t], cv);
    }
    __syncthreads();
    lds_reduce(lds, C, C > 1);  // one chunk: its last block already carried ROOT
    if (t < 8) out[(size_t)r.w * 8 + t] = lds[0][t];
}

// ------------------------------------------------------------------ whole-file cas
// Work items built on the host (sd_cas_api.cpp, plan_whole_items), 16 bytes each:
//   full-pair item  (u64 pair offset, CV slot, first chunk index): an aligned chunk pair
//                   lying wholly inside a message of >= 3 chunks -- 32 full blocks and one
//                   parent, never ROOT; the sampled kernel's branch-free line-pair loop.
//   tail item       (u64 offset, CV slot or file, glen | c0 << 12 | root << 31): a
//                   message's partial last pair, or the whole message when it has <= 2
//                   chunks (then ROOT).  Sorted on the host by compression count, so the
//                   lanes of a wave have equal trip counts.
// Workgroups [0, wf) take full-pair items, the rest tail items (a workgroup-uniform
// branch); the tail path hashes its chunks one after the other without the second message
// buffer, so the kernel keeps the full path's register budget, and its latency-bound
// lanes run while the last full-pair waves drain.
__global__ __launch_bounds__(256) void k_whole_items(const uint8_t* __restrict__ staged,
                                                     const uint4* __restrict__ full, uint32_t n_full, uint32_t wf,
                                                     const uint4* __restrict__ tail, uint32_t n_tail,
                                                     uint32_t* __restrict__ cvbuf, uint32_t* __restrict__ out) {
    if (blockIdx.x < wf) {
        const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
        if (g >= n_full) return;
        const uint4 it = full[g];
        const uint64_t off = (uint64_t)it.x | ((uint64_t)it.y << 32);
        uint32_t cv[8];
        full_chunks_cv<2>(cv, staged + off, it.w);
        store_cv(cvbuf + (size_t)it.z * 8, cv);
        return;
    }
    const uint32_t g = (blockIdx.x - wf) * blockDim.x + threadIdx.x;
    if (g >= n_tail) return;
    const uint4 it = tail[g];
    const uint8_t* p = staged + ((uint64_t)it.x | ((uint64_t)it.y << 32));
    const uint32_t glen = it.w & 0xFFFu, c0 = (it.w >> 12) & 0x7FFFFu;
    const bool root = (it.w >> 31) != 0u;
    uint32_t cv[8];
    if (glen <= CHUNK_LEN) {
        chunk_cv(cv, p, glen, c0, root);
    } else {
        uint32_t l[8], r[8];
        chunk_cv(l, p, CHUNK_LEN, c0, false);
        chunk_cv(r, p + CHUNK_LEN, glen - CHUNK_LEN, c0 + 1, false);
        parent(cv, l, r, root ? ROOT : 0u);
    }
    store_cv((root ? out : cvbuf) + (size_t)it.z * 8, cv);
}

// Item = (first node slot in src, m | root << 31, dst slot or file): merges nodes
// src[first .. first + m), m in 1..8, an aligned group of one file's node list (every node
// but the last a full subtree of one size), into one CV, level-wise (below).  ROOT on the
// final parent when the group is the whole file.  Two passes (<= 8 pair nodes, then <= 8 of
// those) cover messages of up to 128 chunks.  (Round 5: every node loaded up front, 4 %
// faster than merging each into a CV stack as it arrived, profiles/r5/r5w_merge8_trace.md;
// the stack version is in e9a97a5.)
__global__ __launch_bounds__(256) void k_whole_merge8(const uint4* __restrict__ items, uint32_t n,
                                                      const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                      uint32_t* __restrict__ out) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const uint4 it = items[g];
    const uint32_t m = it.y & 0xFu;
    const bool root = (it.y >> 31) != 0u;
    // All m node CVs are loaded at once (they were written by another XCD's workgroups, so
    // each load is a trip past this XCD's L2: one round trip per lane instead of m), then
    // merged level-wise with static register indices -- pairs (2k, 2k+1), the odd node
    // carried up -- the BLAKE3 tree of an aligned group.  The lanes of a wave hold items
    // sorted by node count, so the guarded parents rarely diverge.
    uint32_t nd[8][8];
#pragma unroll
    for (int k = 0; k < 8; k++)
        if ((uint32_t)k < m) load_cv(nd[k], src + (size_t)(it.x + k) * 8);
    uint32_t cnt = m;
#pragma unroll
    for (int lvl = 0; lvl < 3; lvl++) {
        const uint32_t flags = (root && cnt == 2u) ? ROOT : 0u;
#pragma unroll
        for (int k = 0; k < 4 >> lvl; k++) {
            if ((uint32_t)(2 * k + 1) < cnt) {
                uint32_t r[8];
                parent(r, nd[2 * k], nd[2 * k + 1], flags);
#pragma unroll
                for (int i = 0; i < 8; i++) nd[k][i] = r[i];
            } else if ((uint32_t)(2 * k) < cnt) {
#pragma unroll
                for (int i = 0; i < 8; i++) nd[k][i] = nd[2 * k][i];
            }
        }
        cnt = (cnt + 1u) >> 1;
    }
    store_cv((root ? out : dst) + (size_t)it.z * 8, nd[0]);
}

// 32-byte hash rows src[i] -> out[idx[i]] (whole-file cas messages hashed by the checksum
// kernels land in their batch's output order)
__global__ __launch_bounds__(256) void k_scatter_hash(const uint32_t* __restrict__ src, const uint32_t* __restrict__ idx,
                                                      uint32_t n, uint32_t* __restrict__ out) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n * 8u) return;
    out[(size_t)idx[g >> 3] * 8 + (g & 7u)] = src[g];
}

// ------------------------------------------------------------------------ checksums
// Leaf: 1 MiB blocks = 1024 chunks of one message, CK_WG_BLOCKS (2) blocks per workgroup of
// 256 lanes each.  Lane l of a block hashes its chunks [4l, 4l+4) one after the other
// (line-pair loads) and merges them in-lane with the CV stack; then the lane CVs of each
// block merge level-wise in LDS with the blocks' trees packed together: at tree level L the
// parents of both blocks sit in the lowest lanes, so the workgroup's waves run partly masked
// only at the top levels, once per two blocks (round 5: with one block per workgroup its
// 8-level tree left 321 lane-compressions of every 17 728 masked, 1.8 %; two blocks leave
// 129 per block -- 0.3-1.2 % faster, profiles/r5/r5zk_ck_leaf_ab/; 16- or 8-chunk lanes
// with 4 or 2 blocks per 256-lane workgroup lost it again to 4x / 2x longer workgroups, and
// 4 blocks of 256 lanes per workgroup to occupancy, r5zk1 and r5zk).  Block number =
// wg_map[i].y + blk_base for entry i = CK_WG_BLOCKS x workgroup + (lane / 256); `shift` is
// subtracted from the message's byte offset (a streamed window holds message bytes
// [shift, shift + window)).
#ifndef SD_CK_LANE_CHUNKS
#define SD_CK_LANE_CHUNKS 4
#endif
#ifndef SD_CK_WG_BLOCKS
#define SD_CK_WG_BLOCKS 2
#endif
constexpr uint32_t CK_BLOCK_CHUNKS = 1024;
constexpr uint32_t CK_LANE_CHUNKS = SD_CK_LANE_CHUNKS;
constexpr uint32_t CK_BLOCK_LANES = CK_BLOCK_CHUNKS / CK_LANE_CHUNKS;
constexpr uint32_t CK_WG_BLOCKS = SD_CK_WG_BLOCKS;
constexpr uint32_t CK_WG_THREADS = CK_BLOCK_LANES * CK_WG_BLOCKS;
constexpr uint32_t CK_TREE_LEVELS = ilog2(CK_BLOCK_LANES);
static_assert((CK_LANE_CHUNKS & (CK_LANE_CHUNKS - 1)) == 0 && CK_LANE_CHUNKS >= 2 && CK_LANE_CHUNKS <= 16, "lane chunks");
static_assert(CK_WG_THREADS >= 64 && CK_WG_THREADS <= 1024 && CK_WG_THREADS % 64 == 0, "workgroup size");

__global__ __launch_bounds__(CK_WG_THREADS) void k_ck_leaf(
    const uint8_t* __restrict__ data, uint64_t shift, uint32_t blk_base, const ck_file* __restrict__ files,
    const uint2* __restrict__ wg_map, uint32_t n_blocks, uint32_t* __restrict__ cvbuf, uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[CK_WG_THREADS][8];
    __shared__ uint32_t s_lanes[CK_WG_BLOCKS], s_root[CK_WG_BLOCKS];
    __shared__ uint64_t s_dst[CK_WG_BLOCKS];  // output row: file (root) or CV slot, | 1 << 63 for out
    const uint32_t t = threadIdx.x, wv = t / CK_BLOCK_LANES, lane = t % CK_BLOCK_LANES;
    const uint32_t bi = blockIdx.x * CK_WG_BLOCKS + wv;  // this lane's block entry
    uint32_t lanes_b = 0, root_b = 0;
    uint64_t dst_b = 0;
    if (bi < n_blocks) {
        const uint2 wm = wg_map[bi];  // (file, block)
        const uint32_t blk = wm.y + blk_base;
        const ck_file fi = files[wm.x];
        const uint64_t nchunks = fi.len == 0 ? 1 : (fi.len + CHUNK_LEN - 1) / CHUNK_LEN;
        const uint64_t blk0 = (uint64_t)blk * CK_BLOCK_CHUNKS;
        const uint32_t blk_chunks = (uint32_t)(nchunks - blk0 < CK_BLOCK_CHUNKS ? nchunks - blk0 : CK_BLOCK_CHUNKS);
        const bool file_is_block = nchunks <= CK_BLOCK_CHUNKS;
        const bool file_is_lane = nchunks <= CK_LANE_CHUNKS;  // the whole message inside lane 0
        lanes_b = (blk_chunks + CK_LANE_CHUNKS - 1) / CK_LANE_CHUNKS;
        root_b = file_is_block && !file_is_lane;
        dst_b = file_is_block ? ((uint64_t)wm.x | (1ull << 63)) : fi.cv_base + blk;
        const uint32_t c0 = lane * CK_LANE_CHUNKS;
        if (c0 < blk_chunks) {
            const uint32_t nch = blk_chunks - c0 < CK_LANE_CHUNKS ? blk_chunks - c0 : CK_LANE_CHUNKS;
            const uint8_t* p = data + (fi.offset - shift);
            CvStack<ilog2(CK_LANE_CHUNKS)> st;  // after chunk j it holds popcount(j + 1) subtrees
            uint32_t cv[8];
#pragma unroll 1
            for (uint32_t j = 0; j < nch; j++) {
                const uint64_t ci = blk0 + c0 + j;
                const uint64_t rem = fi.len - ci * CHUNK_LEN;
                const uint32_t len = fi.len == 0 ? 0u : (rem < CHUNK_LEN ? (uint32_t)rem : CHUNK_LEN);
                if (len == CHUNK_LEN && nchunks > 1) full_chunk_cv_lp(cv, p + ci * CHUNK_LEN, ci);
                else chunk_cv(cv, p + ci * CHUNK_LEN, len, ci, nchunks == 1);
                if (j + 1 < nch) {  // an aligned group that ends here merges, then waits on the stack
#pragma unroll 1
                    for (uint32_t g = j + 1; (g & 1u) == 0; g >>= 1) st.merge_top(cv, 0u);
                    st.push(cv);
                } else {  // the lane's last chunk: its aligned merges and the fold, one run of
                          // popcount(nch - 1) merges; ROOT on the last when the file is this lane
                    const uint32_t ops = (uint32_t)__builtin_popcount(nch - 1);
#pragma unroll 1
                    for (uint32_t k = ops; k > 0; k--) st.merge_top(cv, (file_is_lane && k == 1) ? ROOT : 0u);
                }
            }
            store_cv(lds[t], cv);
        }
    }
    if (lane == 0) {
        s_lanes[wv] = lanes_b;
        s_root[wv] = root_b;
        s_dst[wv] = dst_b;
    }
    __syncthreads();
    // the blocks' trees, level-wise with the odd node carried up (CK_BLOCK_LANES -> 1); block
    // b's level-L nodes at lds[CK_BLOCK_LANES b .. + n_b(L))
#pragma unroll 1
    for (uint32_t L = 0; L < CK_TREE_LEVELS; L++) {
        const uint32_t P = (CK_BLOCK_LANES / 2) >> L;  // parent slots per block at this level
        uint32_t res[8];
        bool have = false;
        uint32_t to = 0;
        if (t < CK_WG_BLOCKS * P) {
            const uint32_t b = t / P, j = t - b * P;
            uint32_t nb = s_lanes[b];
            for (uint32_t l = 0; l < L; l++) nb = (nb + 1) >> 1;
            if (2 * j + 1 < nb) {
                uint32_t l8[8], r8[8];
                load_cv(l8, lds[CK_BLOCK_LANES * b + 2 * j]);
                load_cv(r8, lds[CK_BLOCK_LANES * b + 2 * j + 1]);
                parent(res, l8, r8, (s_root[b] && nb == 2) ? ROOT : 0u);
                have = true;
            } else if (2 * j + 1 == nb) {  // the odd last node
                load_cv(res, lds[CK_BLOCK_LANES * b + 2 * j]);
                have = true;
            }
            to = CK_BLOCK_LANES * b + j;
        }
        __syncthreads();
        if (have) store_cv(lds[to], res);
        __syncthreads();
    }
    if (t < 8 * CK_WG_BLOCKS) {
        const uint32_t b = t >> 3, w = t & 7u;
        if (s_lanes[b]) {
            const uint64_t d = s_dst[b];
            if (d >> 63) out[(d & ~(1ull << 63)) * 8 + w] = lds[CK_BLOCK_LANES * b][w];
            else cvbuf[d * 8 + w] = lds[CK_BLOCK_LANES * b][w];
        }
    }
}

// Reduce: workgroup = up to 256 consecutive CVs of one message's level; writes one CV to
// the next level, or the root hash when the level fits one group.
__global__ __launch_bounds__(256) void k_ck_reduce(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                   const ck_reduce_wg* __restrict__ wgs, uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[256][8];
    const ck_reduce_wg w = wgs[blockIdx.x];
    const uint32_t t = threadIdx.x;
    if (t < w.count) {
        uint32_t cv[8];
        load_cv(cv, src + (w.src_base + t) * 8);
        store_cv(lds[t], cv);
    }
    __syncthreads();
    lds_reduce(lds, w.count, w.is_root != 0);
    if (t < 8) {
        if (w.is_root) out[(size_t)w.file * 8 + t] = lds[0][t];
        else dst[w.dst_index * 8 + t] = lds[0][t];
    }
}

// --------------------------------------------------------------------- launchers
namespace sdk {

uint64_t cas_sampled_rows_bytes(uint32_t n) { return (uint64_t)n * S_K * 32; }

// rows >= cas_sampled_rows_bytes(n)
hipError_t launch_cas_sampled(const uint8_t* staged, const uint64_t* soff, const uint32_t* idx, uint32_t n,
                              uint32_t* rows, uint32_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t lanes_wg = (uint32_t)(((uint64_t)n * S_K + 255) / 256), merge_wg = (n + 255) / 256;
    hipLaunchKernelGGL(k_cas_sampled_lanes<S_U>, dim3(lanes_wg), dim3(256), 0, s, staged, soff, n, rows);
    hipLaunchKernelGGL(k_cas_sampled_merge<S_U>, dim3(merge_wg), dim3(256), 0, s, staged, soff, idx, n, rows, out);
    return hipGetLastError();
}

hipError_t launch_whole_wave(const uint8_t* staged, const uint4* rows, uint32_t n, uint32_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_whole_wave, dim3(n), dim3(128), 0, s, staged, rows, out);
    return hipGetLastError();
}

hipError_t launch_cas_sampled_wave(const uint8_t* staged, const uint64_t* soff, const uint32_t* idx, uint32_t n,
                                   uint32_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_cas_sampled_wave, dim3(n), dim3(64), 0, s, staged, soff, idx, n, out);
    return hipGetLastError();
}

hipError_t launch_whole_items(const uint8_t* staged, const uint4* full, uint32_t n_full, const uint4* tail,
                              uint32_t n_tail, const uint4* merge_a, uint32_t n_a, const uint4* merge_b, uint32_t n_b,
                              uint32_t* cvbuf, uint32_t* cv2, uint32_t* out, hipStream_t s) {
    const uint32_t wf = (n_full + 255) / 256, wt = (n_tail + 255) / 256;
    if (wf + wt)
        hipLaunchKernelGGL(k_whole_items, dim3(wf + wt), dim3(256), 0, s, staged, full, n_full, wf, tail, n_tail,
                           cvbuf, out);
    if (n_a)
        hipLaunchKernelGGL(k_whole_merge8, dim3((n_a + 255) / 256), dim3(256), 0, s, merge_a, n_a,
                           (const uint32_t*)cvbuf, cv2, out);
    if (n_b)
        hipLaunchKernelGGL(k_whole_merge8, dim3((n_b + 255) / 256), dim3(256), 0, s, merge_b, n_b,
                           (const uint32_t*)cv2, (uint32_t*)nullptr, out);
    return hipGetLastError();
}

hipError_t launch_scatter_hash(const uint32_t* src, const uint32_t* idx, uint32_t n, uint32_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scatter_hash, dim3((n * 8 + 255) / 256), dim3(256), 0, s, src, idx, n, out);
    return hipGetLastError();
}

hipError_t launch_ck_leaf(const uint8_t* data, uint64_t shift, uint32_t blk_base, const ck_file* files,
                          const uint2* wg_map, uint32_t n_wg, uint32_t* cvbuf, uint32_t* out, hipStream_t s) {
    if (n_wg == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ck_leaf, dim3((n_wg + CK_WG_BLOCKS - 1) / CK_WG_BLOCKS), dim3(CK_WG_THREADS), 0, s, data, shift,
                       blk_base, files, wg_map, n_wg, cvbuf, out);
    return hipGetLastError();
}

hipError_t launch_ck_reduce(const uint32_t* src, uint32_t* dst, const ck_reduce_wg* wgs, uint32_t n_wg,
                            uint32_t* out, hipStream_t s) {
    if (n_wg == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ck_reduce, dim3(n_wg), dim3(256), 0, s, src, dst, wgs, out);
    return hipGetLastError();
}

}  // namespace sdk
