// fm3d_mser.hip -- the MSER detector on gfx950.
//
// Reference: DescriptorsMatcher's DetectorType MSER (descriptorsmatcher.cpp:258-272:
// cv::MserFeatureDetector(Delta, MinArea, MaxArea, MaxVariation, MinDiversity, MaxEvolution,
// AreaThreshold, MinMargin, EdgeBlurSize) of OpenCV 2.4.9; on grey images only the first five steer
// the result).  Restated in oracle/orc_mser.c (pointer form, as mser.cpp); this file is an index-based
// statement of the same steps and equals the oracle bit for bit.
//
// MSER's linear-time flood (Nister & Stewenius, as mser.cpp implements it) is one priority flood per
// pass whose visiting order decides which component's history continues at equal-size merges, which
// point list comes first, and the order the regions come out in -- all part of the detector's output.
// It is sequential by construction, so each pass is one lane (the passes of every image in a batch
// run side by side, one workgroup each; the rest of the workgroup builds the grey-level histogram and
// clears the state first).  A lone wave issues one instruction every four cycles and waits on every
// dependent load, so the state is laid out for few instructions and round trips per pixel:
//   * mser.cpp's padded int image (value, visited bit, next direction) is split: each pass's grey
//     values on the same (w + 2) x (h + 2) grid (mser_pad_kernel; read through the scalar cache), the
//     visited bits a bitmap over that grid in LDS (up to kMserLdsBits cells; HBM beyond) with the
//     border pre-marked (no bounds tests), and the next direction in the bucket entry of a pixel
//     pushed back by a descent ({padded pixel + 1 | direction << 28, x | y << 16});
//   * the top entry of every grey-level bucket is cached in LDS, so a pop reads LDS and the refill
//     of that bucket's new top from HBM is issued with the neighbours' value loads;
//   * the top component of the stack stays in registers (size, tail, history), the ones below it in
//     LDS.
// The point lists (node = {next, x | y << 16}) and the histories are in HBM.  After the floods the
// lists are ranked (Wyllie) so every region's points are one contiguous run, and fitEllipse runs one
// wave per region (its three least-squares solves are OpenCV's scalar one-sided Jacobi SVD, every sum
// in the region list's order), all regions in parallel.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "fm3d_detmath.h"
#include "fm3d_kernels.h"

namespace fm3d {

MserLayout mser_layout(int w, int h) {
    MserLayout L;
    L.w = w;
    L.h = h;
    const long long N = (long long)w * h, NP = (long long)(w + 2) * (h + 2);
    L.pw = w + 2;
    L.visInLds = NP <= kMserLdsBits;
    L.visWords = (NP + 31) / 32;
    L.padBytes = (NP + 3) & ~3LL;
    L.heapEntries = N + 256;
    L.nodes = N;
    L.hists = 2 * N + 2;
    L.regCap = N + 1;
    return L;
}

namespace {

struct Comp {  // MSERConnectedComp by index
    int head, tail, hist, level, size, dvar;
    float var;
};

constexpr int kMserThreads = 256;

__device__ __forceinline__ void comp_init(Comp& c) {
    c.size = 0;
    c.var = 0.f;
    c.dvar = 1;
    c.hist = -1;
}

// MSERNewHistory
__device__ __forceinline__ void new_history(Comp& c, MserHist* hist, int hi) {
    MserHist r;
    r.child = hi;
    if (c.hist < 0) {
        r.shortcut = hi;
        r.stable = 0;
    } else {
        hist[c.hist].child = hi;
        r.shortcut = hist[c.hist].shortcut;
        r.stable = hist[c.hist].stable;
    }
    r.val = c.level;
    r.size = c.size;
    hist[hi] = r;
    c.hist = hi;
}

// MSERMergeComp(top, below, below, history): the larger keeps its history (the top one on a tie);
// its point list comes first
// the link of the winner's tail to the other list (tail, head) is returned in `link` (x = -1: none)
__device__ __forceinline__ void merge(const Comp& top, Comp& below, MserHist* hist, int2& link, int hi) {
    const bool topWins = top.size >= below.size;
    const Comp win = topWins ? top : below, lose = topWins ? below : top;
    MserHist r;
    r.child = hi;
    if (win.hist < 0) {
        r.shortcut = hi;
        r.stable = 0;
    } else {
        hist[win.hist].child = hi;
        r.shortcut = hist[win.hist].shortcut;
        r.stable = hist[win.hist].stable;
    }
    if (lose.hist >= 0) {
        const int ls = hist[lose.hist].stable;
        if (ls > r.stable) r.stable = ls;
    }
    r.val = win.level;
    r.size = win.size;
    hist[hi] = r;
    link = (top.size > 0 && below.size > 0) ? make_int2(win.tail, lose.head) : make_int2(-1, 0);
    Comp m;
    m.level = below.level;
    m.var = win.var;
    m.dvar = win.dvar;
    m.head = win.size > 0 ? win.head : lose.head;
    m.tail = lose.size > 0 ? lose.tail : win.tail;
    m.hist = hi;
    m.size = top.size + below.size;
    below = m;
}

// MSERStableCheck (with MSERVariationCalc)
__device__ __forceinline__ bool stable_check(Comp& c, MserHist* hist, const MserParams& P) {
    if (c.hist < 0) return false;
    MserHist H = hist[c.hist];
    if (H.size <= P.minArea || H.size >= P.maxArea) return false;
    const float div = (float)(H.size - H.stable) / (float)H.size;
    int sc = H.shortcut;
    MserHist S = hist[sc];
    while (sc != S.shortcut && S.val + P.delta > c.level) {
        sc = S.shortcut;
        S = hist[sc];
    }
    int ch = S.child;
    MserHist C = hist[ch];
    while (ch != C.child && C.val + P.delta <= c.level) {
        sc = ch;
        S = C;
        ch = C.child;
        C = hist[ch];
    }
    hist[c.hist].shortcut = sc;
    const float var = (float)(c.size - S.size) / (float)S.size;
    const bool dvar = c.var < var || (unsigned)(H.val + 1) < (unsigned)c.level;
    const bool stable = dvar && !c.dvar && (double)c.var < P.maxVariation && (double)div > P.minDiversity;
    c.var = var;
    c.dvar = dvar ? 1 : 0;
    if (stable) hist[c.hist].stable = H.size;
    return stable;
}

// one bucket entry: {pixel + 1 | next direction << 28, x | y << 16}; {0, 0} is a bucket's base
// element i of an 8-byte array through a 32-bit byte offset (the SGPR-base + VGPR-offset address
// form: no 64-bit address arithmetic; every index here is below 2^28)
__device__ __forceinline__ int2& at8(int2* base, int i) { return *(int2*)((uint8_t*)base + ((unsigned)i << 3)); }

// the packed (x | y << 16) step to the neighbour in direction d (right, down, left, up)
constexpr int kStep[4] = {1, 1 << 16, -1, -(1 << 16)};

// each pass's grey values on the padded (w + 2) x (h + 2) grid (pass 0: 255 - I), border 0; the flood
// never reads a border value (the border is marked visited), it only needs no bounds tests
__global__ void mser_pad_kernel(const uint8_t* __restrict__ src, MserLayout L, int slots, uint8_t* pad) {
    const long long NP = (long long)L.pw * (L.h + 2);
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= slots * L.padBytes) return;
    const int slot = (int)(i / L.padBytes), pass = slot & 1;  // slot = 2 * image + pass
    const long long q = i - slot * L.padBytes;
    uint8_t v = 0;
    if (q < NP) {
        const int px = (int)(q % L.pw) - 1, py = (int)(q / L.pw) - 1;
        if (px >= 0 && px < L.w && py >= 0 && py < L.h) {
            const uint8_t g = src[(size_t)(slot >> 1) * L.w * L.h + (size_t)py * L.w + px];
            v = pass == 0 ? (uint8_t)(255 - g) : g;
        }
    }
    pad[i] = v;
}

template <bool LDSVIS>
__global__ __launch_bounds__(kMserThreads) void mser_flood_kernel(const uint8_t* __restrict__ src, MserLayout L,
                                                                   MserParams P, const uint8_t* __restrict__ padAll,
                                                                   unsigned* visAll, int2* heapAll,
                                                                   int2* nodeAll, MserHist* histAll, int4* regAll,
                                                                   int* nreg) {
    const int slot = blockIdx.x, pass = slot & 1, tid = threadIdx.x;  // slot = 2 * image + pass
    const int w = L.w, h = L.h;
    const int N = w * h;
    src += (size_t)(slot >> 1) * N;
    int2* heap = heapAll + (size_t)slot * L.heapEntries;
    int2* node = nodeAll + (size_t)slot * L.nodes;
    MserHist* hist = histAll + (size_t)slot * L.hists;
    int4* reg = regAll + (size_t)slot * L.regCap;
    extern __shared__ unsigned visLds[];
    unsigned* vis = LDSVIS ? visLds : visAll + (size_t)slot * L.visWords;
    __shared__ int hcur[256];
    __shared__ int lsize[256];
    __shared__ int2 topE[257];  // [256]: the no-refill sink
    __shared__ Comp comp[257];
    for (int i = tid; i < 256; i += kMserThreads) lsize[i] = 0;
    for (long long i = tid; i < L.visWords; i += kMserThreads) vis[i] = 0u;
    __syncthreads();
    const unsigned W = (unsigned)L.pw, H = (unsigned)(h + 2);
    for (unsigned i = tid; i < 2 * W + 2 * (H - 2); i += kMserThreads) {  // the border: visited
        const unsigned q = i < W ? i : i < 2 * W ? (H - 1) * W + (i - W) : ((i - 2 * W) / 2 + 1) * W + ((i & 1) ? W - 1 : 0);
        atomicOr(&vis[q >> 5], 1u << (q & 31));
    }
    // preprocessMSER_8UC1's level histogram (pass 0 floods 255 - I, pass 1 I)
    for (int i = tid; i < N; i += kMserThreads) {
        const int g = src[i];
        atomicAdd(&lsize[pass == 0 ? 255 - g : g], 1);
    }
    __syncthreads();
    if (tid != 0) return;
    {
        int base = 0;
        for (int i = 0; i < 256; i++) {
            if (i) base += lsize[i - 1] + 1;
            hcur[i] = base;
            heap[base] = make_int2(0, 0);
            topE[i] = make_int2(0, 0);
        }
    }
    const int color = pass == 0 ? -1 : 1;
    const long long regCap = L.regCap;
    int nnode = 0, nhist = 0, nr = 0;
    // the current pixel: q on the padded grid, xy = x | y << 16 in the image
    unsigned q = W + 1;
    int xy = 0, dir = 0;
    // grey values through the scalar cache (the padded image read as aligned dwords): scalar loads
    // count in lgkmcnt, so they do not wait for the lane's earlier vector stores
    const unsigned* __restrict__ pad4 = (const unsigned*)(padAll + (size_t)slot * L.padBytes);
    int v = (int)((pad4[q >> 2] >> ((q & 3) << 3)) & 255u);
    vis[q >> 5] |= 1u << (q & 31);
    // the stack: comp[1 .. top - 1] in LDS, the top one in T; comp[0] the 256 sentinel
    int top = 1;
    comp[0].level = 256;
    Comp T;
    comp_init(T);
    T.level = v;
    int belowLevel = 256;  // comp[top - 1].level
    // a pop's bucket refill in flight: topE[pendB] = pendE once it has arrived (256: none)
    int pendB = 256;
    int2 pendE = make_int2(0, 0);
    for (;;) {
        // --- the remaining neighbours of p, from direction dir (right, down, left, up) ---
        unsigned np[4];
        int nv[4];
        bool in[4];
#pragma unroll
        for (int d = 0; d < 4; d++) {
            in[d] = d >= dir;  // the padded border is visited: no bounds tests
            np[d] = d == 0 ? q + 1 : d == 1 ? q + W : d == 2 ? q - 1 : q - W;
        }
        // one batch of loads, used unconditionally (none is sunk into a branch)
        unsigned vw[4], gw[4];
#pragma unroll
        for (int d = 0; d < 4; d++) {  // a 32-bit byte offset from the pass's base (the SGPR-offset form)
            const unsigned off = (unsigned)__builtin_amdgcn_readfirstlane((int)(np[d] & ~3u));
            gw[d] = *(const unsigned*)((const uint8_t*)pad4 + off);
        }
#pragma unroll
        for (int d = 0; d < 4; d++) vw[d] = vis[np[d] >> 5];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int d = 0; d < 4; d++) nv[d] = (int)((gw[d] >> ((np[d] & 3) << 3)) & 255u);
        bool cand[4];
#pragma unroll
        for (int d = 0; d < 4; d++) cand[d] = in[d] & !((vw[d] >> (np[d] & 31)) & 1u);
        topE[pendB] = pendE;  // the previous pop's refill (issued before these loads; branch-free)
        pendB = 256;
        int descend = -1;
#pragma unroll
        for (int d = 0; d < 4; d++) {
            if (descend >= 0 || !cand[d]) continue;
            if (LDSVIS) {  // the visited bit: ds_or, no wait (the file is built without the atomic
                           // optimizer, which would wrap a single lane's atomic in a lane election)
                __hip_atomic_fetch_or(&vis[np[d] >> 5], 1u << (np[d] & 31), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {  // a plain store of the word read above; a later neighbour in the same word
                      // stores the word with both bits
                const unsigned nw = vw[d] | (1u << (np[d] & 31));
#pragma unroll
                for (int d2 = d + 1; d2 < 4; d2++)
                    if ((np[d2] >> 5) == (np[d] >> 5)) vw[d2] = nw;
                vis[np[d] >> 5] = nw;
            }
            if (nv[d] < v) {
                descend = d;
            } else {
                const int b = nv[d];
                const int t = hcur[b] + 1;
                hcur[b] = t;
                const int2 e = make_int2((int)(np[d] + 1), xy + kStep[d]);  // mser_entry, direction 0
                at8(heap, t) = e;
                topE[b] = e;
            }
        }
        if (descend >= 0) {
            // push p back (resuming after `descend`) and open a component at the neighbour's level
            const int d = descend;
            const int t = hcur[v] + 1;
            hcur[v] = t;
            const int2 e = make_int2((int)(q + 1) | ((d + 1) << 28), xy);
            at8(heap, t) = e;
            topE[v] = e;
            xy += kStep[d];
            q = np[d];
            v = nv[d];
            dir = 0;
            comp[top] = T;
            belowLevel = T.level;
            top++;
            comp_init(T);
            T.level = v;
            continue;
        }
        // accumulateMSERComp: the finished pixel joins the top component's list
        at8(node, nnode) = make_int2(-1, xy);
        if (T.size > 0)
            at8(node, T.tail).x = nnode;
        else
            T.head = nnode;
        T.tail = nnode;
        T.size++;
        nnode++;
        // the next pixel: this level's bucket, else the next non-empty level
        // the top entry and the height read together (the compiler barrier keeps the height's load
        // here instead of merging it with the level-change path's after the branch)
        int2 e = topE[v];
        int hp = hcur[v];
        asm volatile("" ::: "memory");
        int pv = v;
        if (!e.x) {
            pv = 0;
            for (int i = v + 1; i < 256; i++)
                if (topE[i].x) {
                    pv = i;
                    break;
                }
            if (!pv) break;
            e = topE[pv];
            hp = hcur[pv];
        }
        {
            const int t = hp - 1;
            hcur[pv] = t;
            pendE = at8(heap, t);  // the bucket's next top, consumed after the neighbour loads
            pendB = pv;
        }
        q = (unsigned)(e.x & 0x0fffffff) - 1u;
        dir = (int)((unsigned)e.x >> 28);
        xy = e.y;
        if (pv != v) {
            v = pv;
            if (pv < belowLevel) {
                if (stable_check(T, hist, P)) {
                    if (nr < regCap) reg[nr] = make_int4(color, T.head, hist[T.hist].size, 0);
                    nr++;
                }
                new_history(T, hist, nhist++);
                T.level = pv;
            } else {
                for (;;) {
                    top--;
                    Comp B = comp[top];
                    int2 link;
                    merge(T, B, hist, link, nhist++);
                    if (link.x >= 0) at8(node, link.x).x = link.y;
                    T = B;
                    belowLevel = comp[top - 1].level;
                    if (pv <= T.level) break;
                    if (pv < belowLevel) {
                        if (stable_check(T, hist, P)) {
                            if (nr < regCap) reg[nr] = make_int4(color, T.head, hist[T.hist].size, 0);
                            nr++;
                        }
                        new_history(T, hist, nhist++);
                        T.level = pv;
                        break;
                    }
                }
            }
        }
    }
    nreg[slot] = nr;
}

// ---------------------------------------------------------------- the point lists, ranked
// After the floods every region is a run of some node list (a node's successor changes only while it
// is its list's tail).  Wyllie's list ranking puts every node of every flood (global index
// slot * N + node) at base[end of its list] + (its distance to that end), so a region's points are
// one contiguous, backwards run and fitEllipse reads them in parallel instead of walking the list.
__global__ void mser_rank_init_kernel(const int2* __restrict__ node, int N, int n, int* jump, int* rank, int* last,
                                      int* len, int* pred) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int s = node[i].x;
    const int g = s >= 0 ? s + (i / N) * N : -1;  // the slot's nodes start at slot * N
    jump[i] = g;
    rank[i] = g >= 0 ? 1 : 0;
    last[i] = g >= 0 ? g : i;
    len[i] = 0;
    pred[i] = 0;
}

// pred[j] = 1 for every node with a predecessor (a node has at most one)
__global__ void mser_rank_pred_kernel(const int* __restrict__ jump, int* pred, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && jump[i] >= 0) pred[jump[i]] = 1;
}

__global__ void mser_rank_round_kernel(const int* __restrict__ jIn, const int* __restrict__ rIn,
                                       const int* __restrict__ lIn, int* jOut, int* rOut, int* lOut, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int j = jIn[i];
    if (j >= 0) {
        rOut[i] = rIn[i] + rIn[j];
        lOut[i] = lIn[j];
        jOut[i] = jIn[j];
    } else {
        rOut[i] = rIn[i];
        lOut[i] = lIn[i];
        jOut[i] = -1;
    }
}

// each list's length, written at its end by its head
__global__ void mser_rank_len_kernel(const int* __restrict__ rank, const int* __restrict__ last,
                                     const int* __restrict__ pred, int* len, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && !pred[i]) len[last[i]] = rank[i] + 1;
}

constexpr int kRankScan = 1024;  // items per scan block (256 threads x 4)

__device__ __forceinline__ int block_excl_scan256(int v, int* sh, int& total) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const int a = t >= o ? sh[t - o] : 0;
        __syncthreads();
        sh[t] += a;
        __syncthreads();
    }
    total = sh[255];
    const int r = sh[t] - v;
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(256) void mser_scan_sums_kernel(const int* __restrict__ v, int n, int* sums) {
    __shared__ int sh[256];
    const int b = blockIdx.x * kRankScan + threadIdx.x * 4;
    int c = 0;
    for (int k = 0; k < 4; k++) c += b + k < n ? v[b + k] : 0;
    int tot;
    block_excl_scan256(c, sh, tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void mser_scan_top_kernel(int* sums, int nb) {
    __shared__ int sh[256];
    int carry = 0;
    for (int b0 = 0; b0 < nb; b0 += 256) {
        const int i = b0 + threadIdx.x;
        const int c = i < nb ? sums[i] : 0;
        int tot;
        const int e = block_excl_scan256(c, sh, tot);
        if (i < nb) sums[i] = carry + e;
        carry += tot;
    }
}

__global__ __launch_bounds__(256) void mser_scan_out_kernel(const int* __restrict__ v, int n,
                                                            const int* __restrict__ sums, int* out) {
    __shared__ int sh[256];
    const int b = blockIdx.x * kRankScan + threadIdx.x * 4;
    int f[4], c = 0;
    for (int k = 0; k < 4; k++) {
        f[k] = b + k < n ? v[b + k] : 0;
        c += f[k];
    }
    int tot;
    int o = sums[blockIdx.x] + block_excl_scan256(c, sh, tot);
    for (int k = 0; k < 4; k++) {
        if (b + k < n) out[b + k] = o;
        o += f[k];
    }
}

__global__ void mser_rank_scatter_kernel(const int2* __restrict__ node, const int* __restrict__ rank,
                                         const int* __restrict__ last, const int* __restrict__ base, int* pts,
                                         int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) pts[base[last[i]] + rank[i]] = node[i].y;
}

// lane l's double, on every lane (two v_readlane: the index is wave-uniform)
__device__ __forceinline__ double lane_get(double v, int l) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(b & 0xffffffffLL), l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// s + t[0] + t[1] + ... + t[cnt - 1] in that order (t[l] on lane l), on every lane: the terms go
// through LDS (buf: 64 doubles of the wave's own) and every lane reads them back two at a time
// (broadcast), so a term costs half a read and one add instead of two v_readlane and an add
__device__ __forceinline__ double seq_add(double s, double t, int cnt, double* buf) {
    buf[threadIdx.x & 63] = t;
    const double2* b2 = (const double2*)buf;
    int l = 0;
    for (; l + 16 <= cnt; l += 16) {  // 8 reads in flight, then 16 adds
        double2 v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = b2[(l >> 1) + j];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            s += v[j].x;
            s += v[j].y;
        }
    }
    for (; l < cnt; l++) s += buf[l];
    __builtin_amdgcn_wave_barrier();  // every lane's reads before the next chunk's writes
    return s;
}

// the two sums s0 += t0[l], s1 += t1[l] interleaved, each in lane order (buf: 128 doubles)
__device__ __forceinline__ void seq_add2(double& s0, double& s1, double t0, double t1, int cnt, double* buf) {
    const int lane = threadIdx.x & 63;
    buf[2 * lane] = t0;
    buf[2 * lane + 1] = t1;
    const double2* b2 = (const double2*)buf;
    int l = 0;
    for (; l + 8 <= cnt; l += 8) {
        double2 v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = b2[l + j];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            s0 += v[j].x;
            s1 += v[j].y;
        }
    }
    for (; l < cnt; l++) {
        const double2 v = b2[l];
        s0 += v.x;
        s1 += v.y;
    }
    __builtin_amdgcn_wave_barrier();
}

// cv::solve(A, b, DECOMP_SVD) with At = A^T (n rows of m), b constant (bval): JacobiSVDImpl_ +
// SVBkSbImpl_ by one wave.  The element-wise steps run lane-parallel (lane l takes k = l, l + 64,
// ...); every sum runs over k in order, its terms computed by the lanes and added one by one
// (seq_add), so each sum has the scalar loop's bits.  Every lane holds W, Vt and x.
__device__ void svd_solve_wave(double* At, int m, int n, double bval, double* x, double* buf) {
    const int lane = threadIdx.x & 63;
    double W[5], Vt[25];
    const double eps = DBL_EPSILON * 10;
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int base = 0; base < m; base += 64) {
            const int k = base + lane;
            const double t = k < m ? At[i * m + k] : 0.;
            sd = seq_add(sd, t * t, min(64, m - base), buf);
        }
        W[i] = sd;
        for (int k = 0; k < n; k++) Vt[i * n + k] = 0;
        Vt[i * n + i] = 1;
    }
    const int max_iter = m > 30 ? m : 30;
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed = false;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double* Ai = At + i * m;
                double* Aj = At + j * m;
                double a = W[i], pp = 0, bb = W[j];
                for (int base = 0; base < m; base += 64) {
                    const int k = base + lane;
                    const double t = k < m ? Ai[k] * Aj[k] : 0.;
                    pp = seq_add(pp, t, min(64, m - base), buf);
                }
                if (fabs(pp) <= eps * sqrt(a * bb)) continue;
                pp *= 2;
                const double beta = a - bb, gamma = sqrt(pp * pp + beta * beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = pp / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = pp / (gamma * c * 2);
                }
                a = bb = 0;
                for (int base = 0; base < m; base += 64) {
                    const int k = base + lane;
                    double t0 = 0., t1 = 0.;
                    if (k < m) {
                        const double ai = Ai[k], aj = Aj[k];
                        t0 = c * ai + s * aj;
                        t1 = -s * ai + c * aj;
                        Ai[k] = t0;
                        Aj[k] = t1;
                    }
                    const double q0 = t0 * t0, q1 = t1 * t1;
                    seq_add2(a, bb, q0, q1, min(64, m - base), buf);  // interleaved, each in k order
                }
                W[i] = a;
                W[j] = bb;
                changed = true;
                for (int k = 0; k < n; k++) {
                    const double t0 = c * Vt[i * n + k] + s * Vt[j * n + k];
                    const double t1 = -s * Vt[i * n + k] + c * Vt[j * n + k];
                    Vt[i * n + k] = t0;
                    Vt[j * n + k] = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int base = 0; base < m; base += 64) {
            const int k = base + lane;
            const double t = k < m ? At[i * m + k] : 0.;
            sd = seq_add(sd, t * t, min(64, m - base), buf);
        }
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i];
            W[i] = W[j];
            W[j] = t;
            for (int k = lane; k < m; k += 64) {
                t = At[i * m + k];
                At[i * m + k] = At[j * m + k];
                At[j * m + k] = t;
            }
            for (int k = 0; k < n; k++) {
                t = Vt[i * n + k];
                Vt[i * n + k] = Vt[j * n + k];
                Vt[j * n + k] = t;
            }
        }
    }
    for (int i = 0; i < n; i++) {
        if (W[i] <= DBL_MIN) continue;  // OpenCV's random left vector: unused below
        const double t = 1. / W[i];
        for (int k = lane; k < m; k += 64) At[i * m + k] *= t;
    }
    double threshold = 0;
    for (int i = 0; i < n; i++) x[i] = 0;
    for (int i = 0; i < n; i++) threshold += W[i];
    threshold *= DBL_EPSILON * 2;
    for (int i = 0; i < n; i++) {
        double wi = W[i], s = 0;
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        for (int base = 0; base < m; base += 64) {
            const int k = base + lane;
            const double t = k < m ? At[i * m + k] * bval : 0.;
            s = seq_add(s, t, min(64, m - base), buf);
        }
        s *= wi;
        for (int k = 0; k < n; k++) x[k] = x[k] + s * Vt[i * n + k];
    }
}

__global__ __launch_bounds__(64) void mser_fit_kernel(const int4* __restrict__ reg, int n, MserRank K, long long nodes,
                                                      const long long* __restrict__ off,
                                                      MserLayout L, int2* xyAll, double* scratch, fm3d_keypoint* kp,
                                                      int* flag, float* boxOut) {
    const int r = blockIdx.x, lane = threadIdx.x;  // one wave per region
    __shared__ double sbuf[128];                   // the sequential sums' terms
    if (r >= n) return;
    const int4 R = reg[r];  // {colour, head node, count, slot}
    const int m = R.z;
    int2* xy = xyAll + off[r];
    double* At = scratch + 5 * off[r];
    {  // the region's first m list points: a run of its list, stored backwards from the head's slot
        const long long g = R.y + R.w * nodes;
        const long long start = (long long)K.base[K.last[g]] + K.rank[g];
        for (int k = lane; k < m; k += 64) {
            const int q = K.pts[start - k];
            xy[k] = make_int2(q & 0xffff, (int)((unsigned)q >> 16));
        }
    }
    __threadfence_block();
    __syncthreads();
    // the float centroid (OpenCV: a sequential float sum in region-list order).  Where every partial
    // sum stays below 2^24 (m * the largest coordinate), the integer-valued sums are exact in any
    // order: lane-strided + xor tree.  Otherwise (a wide image with a large region) lane 0 adds the
    // points in list order, as the reference.
    float cx = 0.f, cy = 0.f;
    int cmax = 0;
    for (int k = lane; k < m; k += 64) {
        cx = __fadd_rn(cx, (float)xy[k].x);
        cy = __fadd_rn(cy, (float)xy[k].y);
        cmax = max(cmax, max(xy[k].x, xy[k].y));
    }
    for (int o = 32; o > 0; o >>= 1) {
        cx = __fadd_rn(cx, __shfl_xor(cx, o));
        cy = __fadd_rn(cy, __shfl_xor(cy, o));
        cmax = max(cmax, __shfl_xor(cmax, o));
    }
    if ((long long)m * (long long)cmax >= (1ll << 24)) {
        float sx = 0.f, sy = 0.f;
        if (lane == 0)
            for (int k = 0; k < m; k++) {
                sx = __fadd_rn(sx, (float)xy[k].x);
                sy = __fadd_rn(sy, (float)xy[k].y);
            }
        cx = __shfl(sx, 0);
        cy = __shfl(sy, 0);
    }
    cx = cx / (float)m;
    cy = cy / (float)m;
    for (int k = lane; k < m; k += 64) {
        const float px = __fsub_rn((float)xy[k].x, cx), py = __fsub_rn((float)xy[k].y, cy);
        At[0 * m + k] = -(double)px * (double)px;
        At[1 * m + k] = -(double)py * (double)py;
        At[2 * m + k] = -(double)px * (double)py;
        At[3 * m + k] = px;
        At[4 * m + k] = py;
    }
    double gfp[5], rp[5];
    svd_solve_wave(At, m, 5, 10000.0, gfp, sbuf);
    {
        double A2[4], x2[2];
        A2[0] = 2 * gfp[0];
        A2[1] = A2[2] = gfp[2];
        A2[3] = 2 * gfp[1];
        // b = (gfp[3], gfp[4]) is not constant: the 2 x 2 solve inline
        double W2[2], V2[4];
        {
            // same steps as svd_solve with m = n = 2 and a vector right-hand side
            double* At2 = A2;
            const double eps = DBL_EPSILON * 10;
            for (int i = 0; i < 2; i++) {
                double sd = 0;
                for (int k = 0; k < 2; k++) sd += At2[i * 2 + k] * At2[i * 2 + k];
                W2[i] = sd;
                V2[i * 2] = 0;
                V2[i * 2 + 1] = 0;
                V2[i * 2 + i] = 1;
            }
            for (int iter = 0; iter < 30; iter++) {
                bool changed = false;
                double a = W2[0], pp = 0, bb = W2[1];
                for (int k = 0; k < 2; k++) pp += At2[k] * At2[2 + k];
                if (!(fabs(pp) <= eps * sqrt(a * bb))) {
                    pp *= 2;
                    const double beta = a - bb, gamma = sqrt(pp * pp + beta * beta);
                    double c, s;
                    if (beta < 0) {
                        const double delta = (gamma - beta) * 0.5;
                        s = sqrt(delta / gamma);
                        c = pp / (gamma * s * 2);
                    } else {
                        c = sqrt((gamma + beta) / (gamma * 2));
                        s = pp / (gamma * c * 2);
                    }
                    a = bb = 0;
                    for (int k = 0; k < 2; k++) {
                        const double t0 = c * At2[k] + s * At2[2 + k];
                        const double t1 = -s * At2[k] + c * At2[2 + k];
                        At2[k] = t0;
                        At2[2 + k] = t1;
                        a += t0 * t0;
                        bb += t1 * t1;
                    }
                    W2[0] = a;
                    W2[1] = bb;
                    changed = true;
                    for (int k = 0; k < 2; k++) {
                        const double t0 = c * V2[k] + s * V2[2 + k];
                        const double t1 = -s * V2[k] + c * V2[2 + k];
                        V2[k] = t0;
                        V2[2 + k] = t1;
                    }
                }
                if (!changed) break;
            }
            for (int i = 0; i < 2; i++) {
                double sd = 0;
                for (int k = 0; k < 2; k++) sd += At2[i * 2 + k] * At2[i * 2 + k];
                W2[i] = sqrt(sd);
            }
            if (W2[0] < W2[1]) {
                double t = W2[0];
                W2[0] = W2[1];
                W2[1] = t;
                for (int k = 0; k < 2; k++) {
                    t = At2[k];
                    At2[k] = At2[2 + k];
                    At2[2 + k] = t;
                    t = V2[k];
                    V2[k] = V2[2 + k];
                    V2[2 + k] = t;
                }
            }
            for (int i = 0; i < 2; i++) {
                if (W2[i] <= DBL_MIN) continue;
                const double t = 1. / W2[i];
                for (int k = 0; k < 2; k++) At2[i * 2 + k] *= t;
            }
            const double b2[2] = {gfp[3], gfp[4]};
            double threshold = 0;
            x2[0] = x2[1] = 0;
            threshold += W2[0];
            threshold += W2[1];
            threshold *= DBL_EPSILON * 2;
            for (int i = 0; i < 2; i++) {
                double wi = W2[i], s = 0;
                if (fabs(wi) <= threshold) continue;
                wi = 1 / wi;
                for (int k = 0; k < 2; k++) s += At2[i * 2 + k] * b2[k];
                s *= wi;
                for (int k = 0; k < 2; k++) x2[k] = x2[k] + s * V2[i * 2 + k];
            }
        }
        rp[0] = x2[0];
        rp[1] = x2[1];
    }
    for (int k = lane; k < m; k += 64) {
        const float px = __fsub_rn((float)xy[k].x, cx), py = __fsub_rn((float)xy[k].y, cy);
        At[0 * m + k] = ((double)px - rp[0]) * ((double)px - rp[0]);
        At[1 * m + k] = ((double)py - rp[1]) * ((double)py - rp[1]);
        At[2 * m + k] = ((double)px - rp[0]) * ((double)py - rp[1]);
    }
    double g[3];
    svd_solve_wave(At, m, 3, 1.0, g, sbuf);
    const double min_eps = 1e-6;
    rp[4] = -0.5 * fm3d_atan2(g[2], g[1] - g[0]);
    double t = fm3d_sin(-2.0 * rp[4]);
    if (fabs(t) > fabs(g[2]) * min_eps)
        t = g[2] / t;
    else
        t = g[1] - g[0];
    rp[2] = fabs(g[0] + g[1] - t);
    if (rp[2] > min_eps) rp[2] = sqrt(2.0 / rp[2]);
    rp[3] = fabs(g[0] + g[1] + t);
    if (rp[3] > min_eps) rp[3] = sqrt(2.0 / rp[3]);
    const float bx = __fadd_rn((float)rp[0], cx), by = __fadd_rn((float)rp[1], cy);
    float bw = (float)(rp[2] * 2), bh = (float)(rp[3] * 2), ang = 0.f;
    if (bw > bh) {
        const float tmp = bw;
        bw = bh;
        bh = tmp;
        ang = (float)(90 + rp[4] * 180 / M_PI);
    }
    if (ang < -180) ang = __fadd_rn(ang, 360.f);
    if (ang > 360) ang = __fsub_rn(ang, 360.f);
    const float diam = sqrtf(bh * bw);
    // Rect::contains(Point(cvRound(cx), cvRound(cy))): cvRound of a NaN, an infinity or a value past
    // the int range is INT_MIN (SSE2), never inside; compared as floats (v_cvt_i32 would give 0 for NaN)
    const float rxf = rintf(bx), ryf = rintf(by);
    const bool inside = rxf >= 0.f && rxf < (float)L.w && ryf >= 0.f && ryf < (float)L.h;
    fm3d_keypoint k;
    k.x = bx;
    k.y = by;
    k.size = diam;
    k.angle = -1.f;
    k.response = 0.f;
    k.octave = 0;
    k.class_id = -1;
    if (lane != 0) return;
    kp[r] = k;
    flag[r] = diam > FLT_EPSILON && inside;
    if (boxOut) {
        boxOut[5 * r + 0] = bx;
        boxOut[5 * r + 1] = by;
        boxOut[5 * r + 2] = bw;
        boxOut[5 * r + 3] = bh;
        boxOut[5 * r + 4] = ang;
    }
}

}  // namespace

void launch_mser_flood(const uint8_t* img, int count, const MserLayout& L, const MserParams& P, uint8_t* pad,
                       unsigned* vis, int2* heap, int2* node, MserHist* hist, int4* reg, int* nreg, hipStream_t s) {
    const int slots = 2 * count;
    mser_pad_kernel<<<(unsigned)((slots * L.padBytes + 255) / 256), 256, 0, s>>>(img, L, slots, pad);
    if (L.visInLds) {
        const size_t lds = (size_t)L.visWords * sizeof(unsigned);
        (void)hipFuncSetAttribute((const void*)mser_flood_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        mser_flood_kernel<true><<<slots, kMserThreads, lds, s>>>(img, L, P, pad, vis, heap, node, hist, reg, nreg);
    } else {
        mser_flood_kernel<false><<<slots, kMserThreads, 0, s>>>(img, L, P, pad, vis, heap, node, hist, reg, nreg);
    }
}

size_t mser_rank_bytes(long long nodes, int slots) {
    return (size_t)(10 * slots * nodes + (slots * nodes + kRankScan) / kRankScan + 8) * 4;
}

MserRank launch_mser_rank(const int2* node, long long nodes, int slots, int* work, hipStream_t s) {
    const int n = (int)(slots * nodes), N = (int)nodes;
    int* jr[2][3] = {{work, work + n, work + 2 * n}, {work + 3 * n, work + 4 * n, work + 5 * n}};
    int* len = work + 6 * n;
    int* base = work + 7 * n;
    int* pts = work + 8 * n;
    int* pred = work + 9 * n;
    int* sums = work + 10 * n;
    const int g = (n + 255) / 256;
    mser_rank_init_kernel<<<g, 256, 0, s>>>(node, N, n, jr[0][0], jr[0][1], jr[0][2], len, pred);
    mser_rank_pred_kernel<<<g, 256, 0, s>>>(jr[0][0], pred, n);
    int cur = 0;
    for (long long span = 1; span < nodes; span <<= 1) {  // ceil(log2 N) doublings reach every list's end
        mser_rank_round_kernel<<<g, 256, 0, s>>>(jr[cur][0], jr[cur][1], jr[cur][2], jr[cur ^ 1][0], jr[cur ^ 1][1],
                                                 jr[cur ^ 1][2], n);
        cur ^= 1;
    }
    mser_rank_len_kernel<<<g, 256, 0, s>>>(jr[cur][1], jr[cur][2], pred, len, n);
    const int nb = (n + kRankScan - 1) / kRankScan;
    mser_scan_sums_kernel<<<nb, 256, 0, s>>>(len, n, sums);
    mser_scan_top_kernel<<<1, 256, 0, s>>>(sums, nb);
    mser_scan_out_kernel<<<nb, 256, 0, s>>>(len, n, sums, base);
    mser_rank_scatter_kernel<<<g, 256, 0, s>>>(node, jr[cur][1], jr[cur][2], base, pts, n);
    MserRank K;
    K.rank = jr[cur][1];
    K.last = jr[cur][2];
    K.base = base;
    K.pts = pts;
    return K;
}

void launch_mser_fit(const int4* reg, int n, const MserRank& K, long long nodes, const long long* off,
                     const MserLayout& L, int2* xy, double* scratch, fm3d_keypoint* kp, int* flag, float* box,
                     hipStream_t s) {
    if (n <= 0) return;
    mser_fit_kernel<<<n, 64, 0, s>>>(reg, n, K, nodes, off, L, xy, scratch, kp, flag, box);
}

}  // namespace fm3d
