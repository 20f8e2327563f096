// cas_kernels.hip -- gfx950 kernels for Spacedrive's content-addressing hot path.
//
//   k_cas_sampled   generate_cas_id, size > 102400 (cas.rs:30-58): every message is the
//                   same 57 352 B = 56 full chunks + one 8-byte chunk, so a workgroup of
//                   7 waves hashes 8 files with one lane per full chunk and merges the
//                   8 x 57 chaining values level-wise in LDS.  No work lists.
//   k_whole_leaf    generate_cas_id, size <= 102400 (cas.rs:27-29): one lane per chunk of
//   k_whole_tree    a host-sorted (msg_len descending) file list; single-chunk files end
//                   in the leaf kernel (ROOT on their last block), multi-chunk files are
//                   merged by one lane each, in place, in the chaining-value buffer.
//   k_ck_leaf       file_checksum (hash.rs:10-24): one 256-lane workgroup per 1 MiB of a
//   k_ck_reduce     file, 4 consecutive chunks per lane merged in-lane, 256 lane CVs
//                   merged in LDS; then 256-way LDS reductions over the block CVs.
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
// 448 lanes = 7 waves.  Each lane hashes U consecutive full chunks of one file (an
// aligned group) and merges them in-lane, so a workgroup covers 8U files.  Per file the
// 56/U lane CVs plus the 8-byte tail chunk (node 56/U, message bytes 57344..57351) are
// merged level-wise in LDS; the tail is hashed during the first level by lanes that have
// no parent to compute (the first level always has 224 parents, and an odd node count,
// so the tail is the carried node).
constexpr int S_FULL = 56;       // full chunks per sampled message (57344 bytes)
constexpr int S_THREADS = 448;

template <int U>
struct sampled_lds {
    static constexpr int LANES = S_FULL / U;     // lanes per file
    static constexpr int F = S_THREADS / LANES;  // files per workgroup = 8U
    static constexpr int N0 = LANES + 1;         // nodes per file entering the tree
    uint32_t cvs[F][N0][8];
};

// one workgroup (blockIdx-independent: `wg` is its index among sampled workgroups)
template <int U, int PF>
__device__ __forceinline__ void sampled_wg(uint32_t wg, const uint8_t* __restrict__ staged,
                                           const sd_extent* __restrict__ ext, const uint32_t* __restrict__ idx,
                                           uint32_t n, uint32_t* __restrict__ out, sampled_lds<U>& sh) {
    constexpr int LANES = sampled_lds<U>::LANES;
    constexpr int F = sampled_lds<U>::F;
    constexpr int N0 = sampled_lds<U>::N0;
    auto& cvs = sh.cvs;
    const uint32_t t = threadIdx.x;
    {
        const uint32_t f = t / LANES, j = t % LANES;
        const uint32_t g = wg * F + f;
        if (g < n) {
            const uint8_t* msg = staged + ext[idx[g]].msg_offset;
            uint32_t cv[8];
            full_chunks_cv<U, PF>(cv, msg + (size_t)j * U * CHUNK_LEN, (uint64_t)j * U);
            store_cv(cvs[f][j], cv);
        }
    }
    __syncthreads();
    uint32_t nodes = N0;
#pragma unroll 1
    for (int level = 0; nodes > 1; level++) {
        const uint32_t P = nodes >> 1;
        const bool carry = nodes & 1u;
        uint32_t res[8];
        bool have = false;
        uint32_t ff = 0, p = 0;
        if (t < F * P) {
            ff = t / P; p = t % P;
            uint32_t l[8], r[8];
            load_cv(l, cvs[ff][2 * p]);
            load_cv(r, cvs[ff][2 * p + 1]);
            parent(res, l, r, nodes == 2 ? ROOT : 0u);
            have = true;
        } else if (carry) {
            if (level == 0) {  // lanes [224, 224 + F): the tail chunk (8 bytes, chunk index 56)
                const uint32_t gt = wg * F + (t - F * P);
                if (t < F * P + F && gt < n) {
                    ff = t - F * P; p = P;
                    const uint8_t* msg = staged + ext[idx[gt]].msg_offset;
                    chunk_cv(res, msg + (size_t)S_FULL * CHUNK_LEN, SD_SAMPLED_MSG_LEN - S_FULL * CHUNK_LEN, S_FULL,
                             false);
                    have = true;
                }
            } else if (t >= 256 && t < 256 + F) {  // a wave with no parent work carries the odd node
                ff = t - 256; p = P;
                load_cv(res, cvs[ff][nodes - 1]);
                have = true;
            }
        }
        __syncthreads();
        if (have) store_cv(cvs[ff][p], res);
        __syncthreads();
        nodes = P + (carry ? 1u : 0u);
    }
    if (t < F * 8) {
        const uint32_t ff = t >> 3, w = t & 7;
        const uint32_t gg = wg * F + ff;
        if (gg < n) out[(size_t)idx[gg] * 8 + w] = cvs[ff][0][w];
    }
}

template <int U, int PF>
__global__ __launch_bounds__(S_THREADS) void k_cas_sampled(const uint8_t* __restrict__ staged,
                                                           const sd_extent* __restrict__ ext,
                                                           const uint32_t* __restrict__ idx,
                                                           uint32_t n, uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) sampled_lds<U> sh;
    sampled_wg<U, PF>(blockIdx.x, staged, ext, idx, n, out, sh);
}

// ------------------------------------------------------------------ whole-file groups
// Whole-file messages (cas.rs:27-29), sorted by length (descending) on the host and packed
// into groups of consecutive files whose chunk PAIRS fit 448 lanes.  A lane hashes one
// aligned pair of chunks (2j, 2j+1) and merges it in-lane; each file's pair CVs are then
// merged level-wise in LDS.  Parents of a level are assigned compactly: a block scan of
// the per-file parent counts, and a binary search from lane to file (files with parents
// left are a prefix of the group, because nodes shrink monotonically with length).
constexpr int W_THREADS = 448;

struct whole_lds {
    uint32_t cvs[W_THREADS][8];
    uint32_t off[W_THREADS];    // first lane (= first pair node) of each local file
    uint32_t pp[W_THREADS];     // parent prefix of the current level
    uint32_t nodes[W_THREADS];  // node count of each local file at the current level
    uint32_t file[W_THREADS];   // global file index of each local file
    uint32_t wsum[8];
    uint32_t active;            // local files that still have parents at this level
};

// exclusive prefix over the workgroup's threads (blockDim a multiple of 64, <= 512)
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t* wsum, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (uint32_t k = 0; k < blockDim.x / 64; k++) {
        if (k < w) before += wsum[k];
        tot += wsum[k];
    }
    __syncthreads();
    total = tot;
    return before + x - v;
}

// largest f in [0, cnt) with pref[f] <= t (pref strictly increasing on [0, cnt))
__device__ __forceinline__ uint32_t find_owner(const uint32_t* pref, uint32_t cnt, uint32_t t) {
    uint32_t lo = 0, hi = cnt - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (pref[mid] <= t) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Level-wise merge of a forest held in LDS: local file f (f < cnt, longest first) has
// sh.nodes[f] CVs at sh.cvs[sh.off[f] ...].  Parents of a level are assigned compactly: a
// block scan of the per-file parent counts, and a binary search from lane to file (files
// with parents left are a prefix, since node counts shrink monotonically with length).
// ROOT goes on each file's final parent, whose CV is the hash written to out[file].
// Every thread of the workgroup must call it.
__device__ __forceinline__ void lds_forest(whole_lds& sh, uint32_t cnt, uint32_t* __restrict__ out) {
    const uint32_t t = threadIdx.x;
    uint32_t maxn = sh.nodes[0];  // local file 0 is the longest
#pragma unroll 1
    while (maxn > 1) {
        uint32_t n = 0, P = 0;
        if (t < cnt) {
            n = sh.nodes[t];
            P = n >= 2 ? n / 2 : 0;
            if (P && (t + 1 == cnt || sh.nodes[t + 1] < 2)) sh.active = t + 1;
        }
        uint32_t tp;
        const uint32_t pp = block_exscan(P, sh.wsum, tp);  // its barriers also publish sh.active
        if (t < cnt) sh.pp[t] = pp;
        __syncthreads();
        uint32_t res[8], keep[8];
        bool have = false, root = false, carry = false;
        uint32_t dst = 0, cdst = 0, rfile = 0;
        if (t < tp) {
            const uint32_t f = find_owner(sh.pp, sh.active, t);
            const uint32_t base = sh.off[f], nf = sh.nodes[f], q = t - sh.pp[f];
            uint32_t l[8], r[8];
            load_cv(l, sh.cvs[base + 2 * q]);
            load_cv(r, sh.cvs[base + 2 * q + 1]);
            root = nf == 2;
            parent(res, l, r, root ? ROOT : 0u);
            have = true;
            dst = base + q;
            rfile = sh.file[f];
        }
        if (t < cnt && n >= 3 && (n & 1u)) {  // the odd node is carried up unchanged
            load_cv(keep, sh.cvs[sh.off[t] + n - 1]);
            carry = true;
            cdst = sh.off[t] + n / 2;
        }
        __syncthreads();
        if (have) {
            if (root) store_cv(out + (size_t)rfile * 8, res);
            else store_cv(sh.cvs[dst], res);
        }
        if (carry) store_cv(sh.cvs[cdst], keep);
        if (t < cnt) sh.nodes[t] = (n + 1) / 2;
        __syncthreads();
        maxn = sh.nodes[0];
    }
}

template <bool PAIRPF>
__device__ __forceinline__ void whole_wg(uint32_t g, const uint8_t* __restrict__ staged,
                                         const sd_extent* __restrict__ ext, const uint32_t* __restrict__ order,
                                         const uint2* __restrict__ groups, uint32_t* __restrict__ out,
                                         whole_lds& sh) {
    const uint2 grp = groups[g];  // (first index in the sorted order, file count)
    const uint32_t cnt = grp.y, t = threadIdx.x;
    uint32_t L = 0;
    if (t < cnt) {
        const uint32_t fl = order[grp.x + t];
        const uint32_t C = (ext[fl].msg_len + CHUNK_LEN - 1) / CHUNK_LEN;  // msg_len >= 8
        L = (C + 1) / 2;
        sh.file[t] = fl;
        sh.nodes[t] = L;
    }
    uint32_t lanes;
    const uint32_t o = block_exscan(L, sh.wsum, lanes);
    if (t < cnt) sh.off[t] = o;
    __syncthreads();
    if (t < lanes) {  // leaf: one aligned chunk pair
        const uint32_t f = find_owner(sh.off, cnt, t);
        const uint32_t fl = sh.file[f];
        const sd_extent e = ext[fl];
        const uint32_t C = (e.msg_len + CHUNK_LEN - 1) / CHUNK_LEN;
        const uint32_t c0 = 2 * (t - sh.off[f]);
        const uint8_t* p = staged + e.msg_offset + (size_t)c0 * CHUNK_LEN;
        const uint32_t rem0 = e.msg_len - c0 * CHUNK_LEN;
        uint32_t res[8];
        if (PAIRPF) {
            pair_cv(res, p, rem0 < 2 * CHUNK_LEN ? rem0 : 2 * CHUNK_LEN, c0, C <= 2);
        } else {
            chunk_cv(res, p, rem0 < CHUNK_LEN ? rem0 : CHUNK_LEN, c0, C == 1);
            if (c0 + 1 < C) {
                uint32_t cv1[8], cv0[8];
                const uint32_t rem1 = rem0 - CHUNK_LEN;
#pragma unroll
                for (int i = 0; i < 8; i++) cv0[i] = res[i];
                chunk_cv(cv1, p + CHUNK_LEN, rem1 < CHUNK_LEN ? rem1 : CHUNK_LEN, c0 + 1, false);
                parent(res, cv0, cv1, C == 2 ? ROOT : 0u);
            }
        }
        if (C <= 2) store_cv(out + (size_t)fl * 8, res);
        else store_cv(sh.cvs[t], res);
    }
    __syncthreads();
    lds_forest(sh, cnt, out);
}

// One launch for a whole cas batch: workgroups [0, S) hash sampled files (8U each),
// workgroups [S, S + G) hash whole-file groups.  The long sampled workgroups are
// dispatched first and the shorter whole-file ones fill the tail.
template <int U>
union mixed_lds {
    sampled_lds<U> s;
    whole_lds w;
};

template <int U, int PF, bool PAIRPF>
__global__ __launch_bounds__(S_THREADS) void k_cas_mixed(const uint8_t* __restrict__ staged,
                                                         const sd_extent* __restrict__ ext,
                                                         const uint32_t* __restrict__ sidx, uint32_t n_sampled,
                                                         uint32_t S, const uint32_t* __restrict__ order,
                                                         const uint2* __restrict__ groups,
                                                         uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) mixed_lds<U> sh;
    if (blockIdx.x < S) sampled_wg<U, PF>(blockIdx.x, staged, ext, sidx, n_sampled, out, sh.s);
    else whole_wg<PAIRPF>(blockIdx.x - S, staged, ext, order, groups, out, sh.w);
}

// ------------------------------------------------------------------ whole-file cas
// chunk_prefix[k]: first global chunk of sorted file k (k = 0..nw, prefix[nw] = total).
// hint[w]: sorted file holding chunk 64*w.
__global__ __launch_bounds__(256) void k_whole_leaf(const uint8_t* __restrict__ staged,
                                                    const sd_extent* __restrict__ ext,
                                                    const uint32_t* __restrict__ order,
                                                    const uint32_t* __restrict__ chunk_prefix,
                                                    const uint32_t* __restrict__ hint, uint32_t nw,
                                                    uint32_t total_chunks, uint32_t* __restrict__ cvbuf,
                                                    uint32_t* __restrict__ out) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= total_chunks) return;
    const uint32_t w = g >> 6;
    uint32_t lo = hint[w], hi = hint[w + 1];
    if (hi > nw - 1) hi = nw - 1;
    while (lo < hi) {  // largest k in [lo, hi] with chunk_prefix[k] <= g
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (chunk_prefix[mid] <= g) lo = mid; else hi = mid - 1;
    }
    const uint32_t k = lo;
    const uint32_t file = order[k];
    const uint32_t c = g - chunk_prefix[k];
    const uint32_t C = chunk_prefix[k + 1] - chunk_prefix[k];
    const sd_extent e = ext[file];
    const uint32_t rem = e.msg_len - c * CHUNK_LEN;
    const uint32_t len = rem < CHUNK_LEN ? rem : CHUNK_LEN;
    uint32_t cv[8];
    chunk_cv(cv, staged + e.msg_offset + (size_t)c * CHUNK_LEN, len, c, C == 1);
    if (C == 1) store_cv(out + (size_t)file * 8, cv);
    else store_cv(cvbuf + (size_t)g * 8, cv);
}

// Pair leaf: one lane per aligned chunk PAIR of a whole-file message (pair_prefix[k] =
// first pair of sorted file k, hint[w] = sorted file holding pair 64*w), prefetching
// block q+1 while q compresses and merging the pair in-lane.  Messages of <= 2 chunks end
// here (ROOT inside the lane); longer ones leave one CV per pair for k_whole_tree, which
// then merges half as many nodes as after the one-chunk-per-lane leaf.
__global__ __launch_bounds__(256) void k_whole_pair_leaf(const uint8_t* __restrict__ staged,
                                                         const sd_extent* __restrict__ ext,
                                                         const uint32_t* __restrict__ order,
                                                         const uint32_t* __restrict__ pair_prefix,
                                                         const uint32_t* __restrict__ hint, uint32_t nw,
                                                         uint32_t total_pairs, uint32_t* __restrict__ cvbuf,
                                                         uint32_t* __restrict__ out) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= total_pairs) return;
    const uint32_t w = g >> 6;
    uint32_t lo = hint[w], hi = hint[w + 1];
    if (hi > nw - 1) hi = nw - 1;
    while (lo < hi) {  // largest k in [lo, hi] with pair_prefix[k] <= g
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (pair_prefix[mid] <= g) lo = mid; else hi = mid - 1;
    }
    const uint32_t k = lo;
    const uint32_t file = order[k];
    const uint32_t j = g - pair_prefix[k];
    const bool root = pair_prefix[k + 1] - pair_prefix[k] == 1u;  // <= 2 chunks
    const sd_extent e = ext[file];
    const uint32_t rem = e.msg_len - j * 2u * CHUNK_LEN;
    uint32_t cv[8];
    pair_cv(cv, staged + e.msg_offset + (size_t)j * 2u * CHUNK_LEN, rem < 2u * CHUNK_LEN ? rem : 2u * CHUNK_LEN,
            2ull * j, root);
    if (root) store_cv(out + (size_t)file * 8, cv);
    else store_cv(cvbuf + (size_t)g * 8, cv);
}

// Forest merge after the pair leaf: workgroup g takes consecutive multi-pair files
// (groups[g] = (first sorted index, count), their pair nodes summing to <= 448), copies
// their node CVs -- one contiguous cvbuf range -- into LDS and merges every file's tree
// level-wise with all lanes (lds_forest): the critical path is log2(nodes) parents
// instead of k_whole_tree's nodes - 1 serial ones per lane.
__global__ __launch_bounds__(W_THREADS) void k_whole_forest(const uint32_t* __restrict__ order,
                                                            const uint32_t* __restrict__ pair_prefix,
                                                            const uint2* __restrict__ groups,
                                                            const uint32_t* __restrict__ cvbuf,
                                                            uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) whole_lds sh;
    const uint2 grp = groups[blockIdx.x];
    const uint32_t cnt = grp.y, t = threadIdx.x;
    const uint32_t base = pair_prefix[grp.x];
    const uint32_t total = pair_prefix[grp.x + cnt] - base;
    if (t < cnt) {
        const uint32_t k = grp.x + t;
        sh.file[t] = order[k];
        sh.nodes[t] = pair_prefix[k + 1] - pair_prefix[k];
        sh.off[t] = pair_prefix[k] - base;
    }
    if (t < total) {
        uint32_t cv[8];
        load_cv(cv, cvbuf + (size_t)(base + t) * 8);
        store_cv(sh.cvs[t], cv);
    }
    __syncthreads();
    lds_forest(sh, cnt, out);
}

// one lane per multi-chunk file (sorted files 0..n_multi-1 all have C >= 2)
__global__ __launch_bounds__(256) void k_whole_tree(const uint32_t* __restrict__ order,
                                                    const uint32_t* __restrict__ chunk_prefix, uint32_t n_multi,
                                                    uint32_t* __restrict__ cvbuf, uint32_t* __restrict__ out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_multi) return;
    uint32_t* base = cvbuf + (size_t)chunk_prefix[k] * 8;
    uint32_t n = chunk_prefix[k + 1] - chunk_prefix[k];
    uint32_t res[8];
    while (n > 1) {  // in place: parent p is written after nodes 2p, 2p+1 were read
        const uint32_t P = n >> 1;
        for (uint32_t p = 0; p < P; p++) {
            uint32_t l[8], r[8];
            load_cv(l, base + (size_t)(2 * p) * 8);
            load_cv(r, base + (size_t)(2 * p + 1) * 8);
            parent(res, l, r, n == 2 ? ROOT : 0u);
            if (n != 2) store_cv(base + (size_t)p * 8, res);
        }
        if (n & 1u) {
            uint32_t cv[8];
            load_cv(cv, base + (size_t)(n - 1) * 8);
            store_cv(base + (size_t)P * 8, cv);
        }
        n = P + (n & 1u);
    }
    store_cv(out + (size_t)order[k] * 8, res);
}

// ------------------------------------------------- whole-file work lists (variant 6)
// The pair leaf splits into two launches over host-built item lists, so every wave runs
// lanes of equal trip count:
//   k_whole_full   every aligned chunk pair lying wholly inside a message of >= 3 chunks:
//                  32 full blocks + one parent, never ROOT -- the sampled kernel's
//                  branch-free loop (full_chunks_cv<2, true>).  91 % of configs[1]'s
//                  compressions.  Item = (u64 pair offset, cv slot, first chunk index).
//   k_whole_tail   the other pairs (a message's partial last pair, or the whole message
//                  when it has <= 2 chunks, then ROOT), sorted on the host by compression
//                  count.  Item = (u64 offset, cv slot or file, glen | c0 << 12 | root << 31).
// and the pair-node trees merge in two launches of k_whole_merge8 (aligned groups of up to
// 8 nodes per lane, level-wise in registers): a critical path of <= 7 + 6 serial parents
// where k_whole_tree's longest lane runs nodes - 1 (50 for a 100 KiB file).
__global__ __launch_bounds__(256) void k_whole_full(const uint8_t* __restrict__ staged, const uint4* __restrict__ items,
                                                    uint32_t n, uint32_t* __restrict__ cvbuf) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const uint4 it = items[g];
    const uint64_t off = (uint64_t)it.x | ((uint64_t)it.y << 32);
    uint32_t cv[8];
    full_chunks_cv<2, true>(cv, staged + off, it.w);
    store_cv(cvbuf + (size_t)it.z * 8, cv);
}

__global__ __launch_bounds__(256) void k_whole_tail(const uint8_t* __restrict__ staged, const uint4* __restrict__ items,
                                                    uint32_t n, uint32_t* __restrict__ cvbuf,
                                                    uint32_t* __restrict__ out) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const uint4 it = items[g];
    const uint64_t off = (uint64_t)it.x | ((uint64_t)it.y << 32);
    const uint32_t glen = it.w & 0xFFFu, c0 = (it.w >> 12) & 0x7FFFFu;
    const bool root = (it.w >> 31) != 0u;
    uint32_t cv[8];
    pair_cv(cv, staged + off, glen, c0, root);
    store_cv((root ? out : cvbuf) + (size_t)it.z * 8, cv);
}

// Both lists in one launch: workgroups [0, wf) take full-pair items, the rest tail items
// (a workgroup-uniform branch).  The tail path hashes its chunks one after the other
// without the prefetch buffer, so the kernel keeps the full path's register budget
// (8 waves/SIMD), and its latency-bound lanes run while the last full-pair waves drain.
template <int PF>  // full-pair message loads, as full_chunks_cv (1: prefetch, 2: line pairs)
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
        full_chunks_cv<2, PF>(cv, staged + off, it.w);
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
// src[first .. first + m), m in 1..8, an aligned group of one file's node list, level-wise
// with the odd node carried up; ROOT on the final parent when the group is the whole file.
__global__ __launch_bounds__(256) void k_whole_merge8(const uint4* __restrict__ items, uint32_t n,
                                                      const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                      uint32_t* __restrict__ out) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const uint4 it = items[g];
    const uint32_t m = it.y & 0xFu;
    const bool root = (it.y >> 31) != 0u;
    uint32_t v[8][8];
#pragma unroll
    for (int i = 0; i < 8; i++)
        if ((uint32_t)i < m) load_cv(v[i], src + (size_t)(it.x + i) * 8);
    uint32_t nn = m;
#pragma unroll
    for (int lvl = 0; lvl < 3; lvl++) {
#pragma unroll
        for (int q = 0; q < (4 >> lvl); q++) {
            if ((uint32_t)(2 * q + 1) < nn) {
                uint32_t t[8];
                parent(t, v[2 * q], v[2 * q + 1], (root && nn == 2) ? ROOT : 0u);
#pragma unroll
                for (int i = 0; i < 8; i++) v[q][i] = t[i];
            } else if ((uint32_t)(2 * q) < nn) {
#pragma unroll
                for (int i = 0; i < 8; i++) v[q][i] = v[2 * q][i];
            }
        }
        nn = (nn + 1) >> 1;
    }
    store_cv((root ? out : dst) + (size_t)it.z * 8, v[0]);
}

// ------------------------------------------------------------------------ checksums
// Leaf: workgroup (256 lanes) = 1 MiB block = 1024 chunks of one file; lane l hashes
// chunks [4l, 4l+4) and merges them in-lane; then the lane CVs merge in LDS.
constexpr uint32_t CK_LANE_CHUNKS = 4;
constexpr uint32_t CK_BLOCK_CHUNKS = 1024;

template <bool LP>  // LP: full chunks with line-pair loads (checksum_variant 1)
__global__ __launch_bounds__(256) void k_ck_leaf(const uint8_t* __restrict__ data, uint64_t shift,
                                                 const ck_file* __restrict__ files,
                                                 const uint2* __restrict__ wg_map,
                                                 uint32_t* __restrict__ cvbuf, uint32_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[256][8];
    const uint2 wm = wg_map[blockIdx.x];  // (file, block)
    const ck_file fi = files[wm.x];
    const uint64_t nchunks = fi.len == 0 ? 1 : (fi.len + CHUNK_LEN - 1) / CHUNK_LEN;
    const uint64_t blk0 = (uint64_t)wm.y * CK_BLOCK_CHUNKS;
    const uint64_t blk_chunks64 = nchunks - blk0 < CK_BLOCK_CHUNKS ? nchunks - blk0 : CK_BLOCK_CHUNKS;
    const uint32_t blk_chunks = (uint32_t)blk_chunks64;
    const uint32_t t = threadIdx.x;
    const uint32_t c0 = t * CK_LANE_CHUNKS;
    const bool file_is_lane = nchunks <= CK_LANE_CHUNKS;  // whole file inside lane 0
    if (c0 < blk_chunks) {
        const uint32_t nch = blk_chunks - c0 < CK_LANE_CHUNKS ? blk_chunks - c0 : CK_LANE_CHUNKS;
        const uint8_t* p = data + (fi.offset - shift);  // shift: window start when streaming
        uint32_t acc[8], cv[8], tmp[8];
        for (uint32_t j = 0; j < nch; j++) {
            const uint64_t ci = blk0 + c0 + j;
            const uint64_t rem = fi.len - ci * CHUNK_LEN;
            const uint32_t len = fi.len == 0 ? 0u : (rem < CHUNK_LEN ? (uint32_t)rem : CHUNK_LEN);
            if (len == CHUNK_LEN && !(file_is_lane && nchunks == 1)) {
                if (LP) full_chunk_cv_lp(cv, p + ci * CHUNK_LEN, ci);
                else full_chunk_cv(cv, p + ci * CHUNK_LEN, ci);
            }
            else chunk_cv(cv, p + ci * CHUNK_LEN, len, ci, nchunks == 1);
            // level-wise in-lane merge of up to 4 chunks: ((0,1),(2,3)) or ((0,1),2)
            if (j == 0) {
#pragma unroll
                for (int i = 0; i < 8; i++) acc[i] = cv[i];
            } else if (j == 1) {
                const bool root = file_is_lane && nch == 2;
                parent(tmp, acc, cv, root ? ROOT : 0u);
#pragma unroll
                for (int i = 0; i < 8; i++) acc[i] = tmp[i];
            } else if (j == 2) {
                if (nch == 3) {
                    parent(tmp, acc, cv, file_is_lane ? ROOT : 0u);
#pragma unroll
                    for (int i = 0; i < 8; i++) acc[i] = tmp[i];
                } else {
#pragma unroll
                    for (int i = 0; i < 8; i++) tmp[i] = cv[i];  // hold chunk 2
                }
            } else {
                uint32_t p23[8];
                parent(p23, tmp, cv, 0u);
                parent(tmp, acc, p23, file_is_lane ? ROOT : 0u);
#pragma unroll
                for (int i = 0; i < 8; i++) acc[i] = tmp[i];
            }
        }
        store_cv(lds[t], acc);
    }
    __syncthreads();
    const uint32_t lanes = (blk_chunks + CK_LANE_CHUNKS - 1) / CK_LANE_CHUNKS;
    const bool file_is_block = nchunks <= CK_BLOCK_CHUNKS;
    lds_reduce(lds, lanes, file_is_block && !file_is_lane);
    if (t < 8) {
        if (file_is_block) out[(size_t)wm.x * 8 + t] = lds[0][t];
        else cvbuf[(fi.cv_base + wm.y) * 8 + t] = lds[0][t];
    }
}

// Reduce: workgroup = up to 256 consecutive CVs of one file's level; writes one CV to the
// next level, or the root hash when the level fits one group.
__global__ __launch_bounds__(256) void k_ck_reduce(const uint32_t* __restrict__ src,
                                                   uint32_t* __restrict__ dst,
                                                   const ck_reduce_wg* __restrict__ wgs,
                                                   uint32_t* __restrict__ out) {
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

hipError_t launch_cas_sampled(const uint8_t* staged, const sd_extent* ext, const uint32_t* idx, uint32_t n,
                              uint32_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int v = tuning_get(SD_TUNE_SAMPLED_VARIANT);
#define SD_LAUNCH_SAMPLED(U, PF)                                                                        \
    hipLaunchKernelGGL((k_cas_sampled<U, PF>), dim3((n + 8 * U - 1) / (8 * U)), dim3(S_THREADS), 0, s, staged, \
                       ext, idx, n, out)
    switch (v) {
        case 10: SD_LAUNCH_SAMPLED(1, false); break;
        case 11: SD_LAUNCH_SAMPLED(1, true); break;
        case 20: SD_LAUNCH_SAMPLED(2, false); break;
        case 21: SD_LAUNCH_SAMPLED(2, 1); break;
        case 22: SD_LAUNCH_SAMPLED(2, 2); break;
        case 12: SD_LAUNCH_SAMPLED(1, 2); break;
        case 42: SD_LAUNCH_SAMPLED(4, 2); break;
        case 40: SD_LAUNCH_SAMPLED(4, false); break;
        default: SD_LAUNCH_SAMPLED(4, true); break;
    }
#undef SD_LAUNCH_SAMPLED
    return hipGetLastError();
}

hipError_t launch_cas_mixed(const uint8_t* staged, const sd_extent* ext, const uint32_t* sidx, uint32_t n_sampled,
                            const uint32_t* order, const uint2* groups, uint32_t n_groups, uint32_t* out,
                            hipStream_t s, bool pairpf) {
    const int v = tuning_get(SD_TUNE_SAMPLED_VARIANT);
#define SD_LAUNCH_MIXED(U, PF, W)                                                                          \
    do {                                                                                                  \
        const uint32_t S = (n_sampled + 8 * U - 1) / (8 * U);                                             \
        if (S + n_groups)                                                                                 \
            hipLaunchKernelGGL((k_cas_mixed<U, PF, W>), dim3(S + n_groups), dim3(S_THREADS), 0, s, staged, \
                               ext, sidx, n_sampled, S, order, groups, out);                              \
    } while (0)
    if (pairpf) {
        switch (v) {
            case 10: SD_LAUNCH_MIXED(1, false, true); break;
            case 11: SD_LAUNCH_MIXED(1, true, true); break;
            case 20: SD_LAUNCH_MIXED(2, false, true); break;
            case 40: SD_LAUNCH_MIXED(4, false, true); break;
            case 41: SD_LAUNCH_MIXED(4, true, true); break;
            default: SD_LAUNCH_MIXED(2, true, true); break;
        }
    } else {
        switch (v) {
            case 10: SD_LAUNCH_MIXED(1, false, false); break;
            case 11: SD_LAUNCH_MIXED(1, true, false); break;
            case 20: SD_LAUNCH_MIXED(2, false, false); break;
            case 40: SD_LAUNCH_MIXED(4, false, false); break;
            case 41: SD_LAUNCH_MIXED(4, true, false); break;
            default: SD_LAUNCH_MIXED(2, true, false); break;
        }
    }
#undef SD_LAUNCH_MIXED
    return hipGetLastError();
}

hipError_t launch_whole_forest(const uint32_t* order, const uint32_t* pair_prefix, const uint2* groups,
                               uint32_t n_groups, const uint32_t* cvbuf, uint32_t* out, hipStream_t s) {
    if (n_groups == 0) return hipSuccess;
    hipLaunchKernelGGL(k_whole_forest, dim3(n_groups), dim3(W_THREADS), 0, s, order, pair_prefix, groups, cvbuf, out);
    return hipGetLastError();
}

hipError_t launch_whole_pair_leaf(const uint8_t* staged, const sd_extent* ext, const uint32_t* order,
                                  const uint32_t* pair_prefix, const uint32_t* hint, uint32_t nw, uint32_t total_pairs,
                                  uint32_t* cvbuf, uint32_t* out, hipStream_t s) {
    if (nw == 0) return hipSuccess;
    hipLaunchKernelGGL(k_whole_pair_leaf, dim3((total_pairs + 255) / 256), dim3(256), 0, s, staged, ext, order,
                       pair_prefix, hint, nw, total_pairs, cvbuf, out);
    return hipGetLastError();
}

hipError_t launch_whole_leaf(const uint8_t* staged, const sd_extent* ext, const uint32_t* order,
                             const uint32_t* chunk_prefix, const uint32_t* hint, uint32_t nw, uint32_t total_chunks,
                             uint32_t* cvbuf, uint32_t* out, hipStream_t s) {
    if (nw == 0) return hipSuccess;
    hipLaunchKernelGGL(k_whole_leaf, dim3((total_chunks + 255) / 256), dim3(256), 0, s, staged, ext, order,
                       chunk_prefix, hint, nw, total_chunks, cvbuf, out);
    return hipGetLastError();
}

hipError_t launch_whole_tree(const uint32_t* order, const uint32_t* chunk_prefix, uint32_t n_multi, uint32_t* cvbuf,
                             uint32_t* out, hipStream_t s) {
    if (n_multi == 0) return hipSuccess;
    hipLaunchKernelGGL(k_whole_tree, dim3((n_multi + 255) / 256), dim3(256), 0, s, order, chunk_prefix, n_multi,
                       cvbuf, out);
    return hipGetLastError();
}

hipError_t launch_whole(const uint8_t* staged, const sd_extent* ext, const uint32_t* order,
                        const uint32_t* chunk_prefix, const uint32_t* hint, uint32_t nw, uint32_t total_chunks,
                        uint32_t n_multi, uint32_t* cvbuf, uint32_t* out, hipStream_t s) {
    if (nw == 0) return hipSuccess;
    hipLaunchKernelGGL(k_whole_leaf, dim3((total_chunks + 255) / 256), dim3(256), 0, s, staged, ext, order,
                       chunk_prefix, hint, nw, total_chunks, cvbuf, out);
    if (n_multi)
        hipLaunchKernelGGL(k_whole_tree, dim3((n_multi + 255) / 256), dim3(256), 0, s, order, chunk_prefix,
                           n_multi, cvbuf, out);
    return hipGetLastError();
}

hipError_t launch_whole_items(const uint8_t* staged, const uint4* full, uint32_t n_full, const uint4* tail,
                              uint32_t n_tail, const uint4* merge_a, uint32_t n_a, const uint4* merge_b, uint32_t n_b,
                              uint32_t* cvbuf, uint32_t* cv2, uint32_t* out, hipStream_t s, bool combined, int pf) {
    if (combined) {
        const uint32_t wf = (n_full + 255) / 256, wt = (n_tail + 255) / 256;
        const size_t lds = (size_t)tuning_get(SD_TUNE_WHOLE_LDS_KB) << 10;
        if (wf + wt && pf == 2)
            hipLaunchKernelGGL(k_whole_items<2>, dim3(wf + wt), dim3(256), lds, s, staged, full, n_full, wf, tail,
                               n_tail, cvbuf, out);
        else if (wf + wt)
            hipLaunchKernelGGL(k_whole_items<1>, dim3(wf + wt), dim3(256), lds, s, staged, full, n_full, wf, tail,
                               n_tail, cvbuf, out);
    } else {
        if (n_full)
            hipLaunchKernelGGL(k_whole_full, dim3((n_full + 255) / 256), dim3(256), 0, s, staged, full, n_full, cvbuf);
        if (n_tail)
            hipLaunchKernelGGL(k_whole_tail, dim3((n_tail + 255) / 256), dim3(256), 0, s, staged, tail, n_tail,
                               cvbuf, out);
    }
    if (n_a)
        hipLaunchKernelGGL(k_whole_merge8, dim3((n_a + 255) / 256), dim3(256), 0, s, merge_a, n_a,
                           (const uint32_t*)cvbuf, cv2, out);
    if (n_b)
        hipLaunchKernelGGL(k_whole_merge8, dim3((n_b + 255) / 256), dim3(256), 0, s, merge_b, n_b,
                           (const uint32_t*)cv2, (uint32_t*)nullptr, out);
    return hipGetLastError();
}

hipError_t launch_ck_leaf(const uint8_t* data, uint64_t shift, const ck_file* files, const uint2* wg_map,
                          uint32_t n_wg, uint32_t* cvbuf, uint32_t* out, hipStream_t s) {
    if (n_wg == 0) return hipSuccess;
    if (tuning_get(SD_TUNE_CK_VARIANT) == 1)
        hipLaunchKernelGGL(k_ck_leaf<true>, dim3(n_wg), dim3(256), 0, s, data, shift, files, wg_map, cvbuf, out);
    else
        hipLaunchKernelGGL(k_ck_leaf<false>, dim3(n_wg), dim3(256), 0, s, data, shift, files, wg_map, cvbuf, out);
    return hipGetLastError();
}

hipError_t launch_ck_reduce(const uint32_t* src, uint32_t* dst, const ck_reduce_wg* wgs, uint32_t n_wg,
                            uint32_t* out, hipStream_t s) {
    if (n_wg == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ck_reduce, dim3(n_wg), dim3(256), 0, s, src, dst, wgs, out);
    return hipGetLastError();
}

}  // namespace sdk
