// fm3d_match.hip -- brute-force k=2 matching + NNDR on gfx950.
//
// Reference: DescriptorsMatcher::compareWithNNDR (descriptorsmatcher.cpp:107-131)
// = knnMatch(A, B, matches, 2) then keep m[0] iff m[0].distance <= eps*m[1].distance.
// The reference's FlannBasedMatcher is approximate (randomised kd-tree / LSH);
// the parity contract is the exact brute force it approximates, ordered by
// (distance, trainIdx) -- SURVEY.md §0 D1.
//
// Three kernels:
//   u8   -- SIFT-like byte rows.  d2 = sum (a-b)^2 = |a'|^2 + |b'|^2 - 2 a'.b' with
//           a' = a - 128 (int8): the dot products run on int8 MFMA
//           (v_mfma_i32_32x32x32_i8, exact int32), the top-2 on the VALU.
//   f32  -- float rows in FLANN's L2 accumulation order (groups of four), VALU.
//   bits -- binary strings, Hamming by popcount, VALU.
#include <hip/hip_runtime.h>

#include <type_traits>
#include <limits.h>
#include <stdlib.h>
#include <stdint.h>

#include "fm3d_kernels.h"

namespace fm3d {

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kQ = 128;     // queries per workgroup (4 waves x 32)
constexpr int kT = 128;     // train rows per LDS tile
constexpr int kThreads = 256;
// 32-query groups per wave of the u8 kernel at 128-byte rows (knn2_i8_kernel's QG): 2 = 200 VGPRs,
// two waves per SIMD; 100k x 100k 2.00 -> 1.85 ms, 10k x 10k 30.7 -> 29.6 us against QG 1 (150
// VGPRs, three waves).  The 256-byte and binary variants keep 1 (a second group would spill).
#ifndef FM3D_KNN_QG
#define FM3D_KNN_QG 2
#endif
constexpr int kQG128 = FM3D_KNN_QG;

__device__ inline int swz_chunk(int row, int ch) {
    // 16-byte chunk XOR swizzle inside each 128-byte segment: rows r..r+15 reading
    // the same logical chunk hit 16 distinct 16-byte bank slots (ds_read_b128).
    return (ch & ~7) | ((ch & 7) ^ ((row >> 1) & 7));
}

// lexicographic (key, idx) top-2 insertion, candidates arriving in increasing idx
__device__ inline void top2_insert(int s, int j, int& b1, int& i1, int& b2, int& i2) {
    bool lt1 = s < b1;
    bool lt2 = s < b2;
    b2 = lt1 ? b1 : (lt2 ? s : b2);
    i2 = lt1 ? i1 : (lt2 ? j : i2);
    b1 = lt1 ? s : b1;
    i1 = lt1 ? j : i1;
}

__device__ inline bool lex_lt(int a, int ia, int b, int ib) {
    return a < b || (a == b && (unsigned)ia < (unsigned)ib);
}

// merge two sorted top-2 lists (a1 <= a2, c1 <= c2 lexicographically); -1 indices sort last
__device__ inline void top2_merge(int& b1, int& i1, int& b2, int& i2, int c1, int j1, int c2, int j2) {
    if (lex_lt(b1, i1, c1, j1)) {
        // best = b1; second = min(b2, c1)
        if (!lex_lt(b2, i2, c1, j1)) {
            b2 = c1;
            i2 = j1;
        }
    } else {
        // best = c1; second = min(b1, c2)
        int nb2 = b1, ni2 = i1;
        if (lex_lt(c2, j2, nb2, ni2)) {
            nb2 = c2;
            ni2 = j2;
        }
        b1 = c1;
        i1 = j1;
        b2 = nb2;
        i2 = ni2;
    }
}

// Ranking keys of the int8 kernel are packed per train tile into one u32 so that the top-2 of a
// tile costs three VALU operations per distance (v_lshl_add_u32, v_max_u32, v_med3_u32).  The
// kernel keeps the LARGEST packed values:
//   bits 31..7: X = kKeyBias - s, s = |b'|^2 - 2 a'.b' (u8) or popc(b) - a.b' (bits); 1 <= X < 2^25
//   bits  6..0: 127 - (row inside its 128-row tile)   (equal s -> the lower row wins)
// The packed row constant ctq = ((kKeyBias - c) << 7) | (127 - row) is formed once per train row;
// the epilogue adds acc << 8 (u8: 2 a'.b') or acc << 7 (bits) to it.  0 marks "no row".
constexpr uint32_t kKeyBias = (1u << 24) + (1u << 22) + 1;  // s in [-2^22, 2^24 + 2^22)
// 128-byte u8 rows (SIFT) in 256-row tiles: eight row bits.  There |b'|^2 <= 2^21 and |2 a'.b'| <= 2^22,
// so s lies in [-2^22, 2^21 + 2^22] and X = kKeyBias8 - s in [1, 2^23 + 2^21 + 1]: 24 bits
constexpr uint32_t kKeyBias8 = (1u << 22) + (1u << 21) + 1;
// train rows per LDS tile of the u8 kernel at 128-byte rows: 256 (one merge, one barrier and one
// staging round per 256 rows; FM3D_KNN_TR256=0 keeps kT)
#ifndef FM3D_KNN_TR256
#define FM3D_KNN_TR256 1
#endif
constexpr int kTR128 = FM3D_KNN_TR256 ? 256 : 128;

__device__ inline uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ inline uint32_t umax(uint32_t a, uint32_t b) { return a < b ? b : a; }
// (plain C, not inline asm, where it reads an MFMA result: the hazard recognizer does not pad
// reads inside asm)
__device__ inline uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) { return umax(umin(a, b), umin(umax(a, b), c)); }
__device__ inline uint32_t pack_row(uint32_t c, int r) { return ((kKeyBias - c) << 7) | (uint32_t)(127 - (r & 127)); }
__device__ inline uint32_t pack_row8(uint32_t c, int r) { return ((kKeyBias8 - c) << 8) | (uint32_t)(255 - (r & 255)); }

// per-row constants of both sides in one launch, 16 bytes per lane (v_dot4_i32_i8 of x' = x - 128
// with itself), lanes of a row summed by shuffles: |x'|^2 for the query rows (cq), the packed
// ranking constant for the train rows (ctp).  Padding bytes are 128 (x' = 0).
__global__ void rowconst_u8_kernel(const uint8_t* __restrict__ A, int nA, const uint8_t* __restrict__ B, int nB,
                                   int dimPad, int* __restrict__ cq, int* __restrict__ ctp, int rowBits) {
    const int cpr = dimPad / 16;  // 8 or 16 lanes per row (power of two)
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int r = t / cpr, k = t - r * cpr;
    const bool isA = r < nA;
    const int rr = isA ? r : r - nA;
    int s = 0;
    if (r < nA + nB) {
        const v4i x = *(const v4i*)((isA ? A : B) + (size_t)rr * dimPad + 16 * k) ^
                      (v4i){(int)0x80808080, (int)0x80808080, (int)0x80808080, (int)0x80808080};
#pragma unroll
        for (int w = 0; w < 4; w++) s = __builtin_amdgcn_sdot4(x[w], x[w], s, false);
    }
    for (int o = 1; o < cpr; o <<= 1) s += __shfl_xor(s, o);
    if (k == 0 && r < nA + nB) {
        if (isA)
            cq[rr] = s;
        else
            ctp[rr] = (int)(rowBits == 8 ? pack_row8((uint32_t)s, rr) : pack_row((uint32_t)s, rr));
    }
}

// binary rows (32 bytes) of both sides unpacked in one launch to int8 rows of 256 bits for the
// MFMA kernel: the query side as 0/1, the train side as -1/+1 (so that popc(b) - a.b' is the Hamming
// distance) with the packed ranking constant popc(b)
__global__ void unpack_bits_kernel(const uint32_t* __restrict__ A, int nA, const uint32_t* __restrict__ B, int nB,
                                   int8_t* __restrict__ outA, int8_t* __restrict__ outB, int* __restrict__ ctp) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;  // one 32-bit word per thread, 8 per row
    const int r = t >> 3, w = t & 7;
    if (r >= nA + nB) return;
    const bool train = r >= nA;
    const int rr = train ? r - nA : r;
    const uint32_t x = (train ? B : A)[(size_t)rr * 8 + w];
    const int lo = train ? -1 : 0;
    int8_t b[32];
#pragma unroll
    for (int k = 0; k < 32; k++) b[k] = ((x >> k) & 1u) ? 1 : lo;
    v4i* o = (v4i*)((train ? outB : outA) + (size_t)rr * 256 + 32 * w);
    o[0] = *(const v4i*)&b[0];
    o[1] = *(const v4i*)&b[16];
    int pc = __popc(x);
    pc += __shfl_xor(pc, 1);
    pc += __shfl_xor(pc, 2);
    pc += __shfl_xor(pc, 4);
    if (train && w == 0) ctp[rr] = (int)pack_row((uint32_t)pc, rr);
}

// KS: dimPad / 32 when it is 4 (128-byte rows) or 8 (256), so the MFMA chain is straight-line
// code; 0 reads it from dimPad.  BITS: rows are pre-unpacked int8 bits (no -128 offset, key
// popc(b) - a.b', no query constant).  QG: 32-query groups per wave (a workgroup holds kQ * QG
// queries); each A fragment read from LDS feeds QG MFMAs, and the per-tile staging, barrier and
// merge are shared by QG groups.
template <int KS, bool BITS, int QG, int TR = kT>
__global__ __launch_bounds__(kThreads) void knn2_i8_kernel(const uint8_t* __restrict__ A, int nA,
                                                           const uint8_t* __restrict__ B, int nB, int dimPad,
                                                           const int* __restrict__ cqA, const int* __restrict__ ctB,
                                                           int tilesPerPart, int* __restrict__ idxOut,
                                                           int* __restrict__ keyOut) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    static_assert(TR == 128 || (TR == 256 && KS == 4 && !BITS), "256-row tiles: 128-byte u8 rows only");
    constexpr int kRB = TR == 256 ? 8 : 7;                 // row bits of a packed key
    constexpr uint32_t kRowMask = (1u << kRB) - 1;
    constexpr uint32_t kBias = TR == 256 ? kKeyBias8 : kKeyBias;
    const int tileBytes = TR * (KS ? 32 * KS : dimPad);
    unsigned char* tiles = smem;                              // 2 x tileBytes
    uint32_t* ctl = (uint32_t*)(smem + 2 * (size_t)tileBytes);  // 2 x TR packed row constants
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int q0 = blockIdx.x * (kQ * QG) + wave * 32 * QG;
    const int half = lane >> 5;
    const int ksteps = KS ? KS : dimPad / 32;
    const int rowBytes = KS ? 32 * KS : dimPad;  // = dimPad (compile-time for KS != 0)
    const int chunksPerRow = rowBytes / 16;
    constexpr int kFlip = BITS ? 0 : (int)0x80808080;  // x ^ 0x80 == x - 128
    constexpr int kShift = BITS ? kRB : kRB + 1;         // acc * MUL << kRB (key bits start at bit kRB)

    // B operand: this lane's query bytes as int8, one set per query group
    v4i bq[QG][8];  // up to dimPad = 256
#pragma unroll
    for (int g = 0; g < QG; g++) {
        const int qrow = q0 + 32 * g + (lane & 31);
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            if (kk < ksteps) {
                v4i v = {0, 0, 0, 0};
                if (qrow < nA) v = *(const v4i*)(A + (size_t)qrow * dimPad + 32 * kk + 16 * half);
                bq[g][kk] = v ^ (v4i){kFlip, kFlip, kFlip, kFlip};
            }
        }
    }
    int b1[QG], i1[QG], b2[QG], i2[QG];
#pragma unroll
    for (int g = 0; g < QG; g++) {
        b1[g] = b2[g] = INT_MAX;
        i1[g] = i2[g] = -1;
    }
    // train tiles of this part (blockIdx.y): [tBeg, tEnd); the parts' lists are merged by knn2_int_merge
    const int tBeg = blockIdx.y * tilesPerPart;
    const int tEnd = min((nB + TR - 1) / TR, tBeg + tilesPerPart);

    // train tiles: the global loads of tile t + 1 are issued into registers before tile t is
    // computed and written to LDS after it, so their latency overlaps the MFMA work
    constexpr int kPre = 8;  // 16-byte chunks per thread and tile (TR * rowBytes / 16 / kThreads at most)
    const int total = TR * chunksPerRow;
    v4i pre[kPre];
    uint32_t preCt = 0;
    auto load_tile = [&](int t) {
        // rows past nB only in the last tile: the others load without a per-chunk test
        const uint8_t* tb = B + (size_t)t * TR * rowBytes;
        if ((t + 1) * TR <= nB) {
#pragma unroll
            for (int i = 0; i < kPre; i++) {
                const int c = tid + i * kThreads;
                if (c < total) pre[i] = *(const v4i*)(tb + (size_t)c * 16);
            }
        } else {
#pragma unroll
            for (int i = 0; i < kPre; i++) {
                const int c = tid + i * kThreads;
                v4i v = {0, 0, 0, 0};
                if (c < total && t * TR + c / chunksPerRow < nB) v = *(const v4i*)(tb + (size_t)c * 16);
                pre[i] = v;
            }
        }
        if (tid < TR) {
            const int j = t * TR + tid;
            preCt = (j < nB) ? (uint32_t)ctB[j] : 0u;
        }
    };
    auto store_tile = [&](int buf) {
        unsigned char* dst = tiles + (size_t)buf * tileBytes;
#pragma unroll
        for (int i = 0; i < kPre; i++) {
            const int c = tid + i * kThreads;
            if (c < total) {
                const int row = c / chunksPerRow, ch = c - row * chunksPerRow;
                *(v4i*)(dst + (size_t)row * rowBytes + 16 * swz_chunk(row, ch)) =
                    pre[i] ^ (v4i){kFlip, kFlip, kFlip, kFlip};
            }
        }
        if (tid < TR) ctl[buf * TR + tid] = preCt;
    };
    struct Acc {
        v16i a[QG];
    };

    if (tBeg < tEnd) {
        load_tile(tBeg);
        store_tile(0);
    }
    __syncthreads();
    for (int t = tBeg; t < tEnd; t++) {
        const int buf = (t - tBeg) & 1;
        if (t + 1 < tEnd) load_tile(t + 1);
        const unsigned char* tl = tiles + (size_t)buf * tileBytes;
        const uint32_t* ct = ctl + buf * TR;
        // packed top-2 (largest) of this tile per query group, two chains (even / odd row blocks)
        // merged after the tile
        uint32_t p1[QG][2], p2[QG][2];
#pragma unroll
        for (int g = 0; g < QG; g++) p1[g][0] = p1[g][1] = p2[g][0] = p2[g][1] = 0;
        // software pipeline over the four 32-row blocks: the MFMA chain of block rb + 1 is issued
        // between the epilogue instructions of block rb (both in flight in one wave)
        auto mma = [&](int rb) {
            Acc acc;
#pragma unroll
            for (int g = 0; g < QG; g++) acc.a[g] = (v16i){0};
            const int arow = rb * 32 + (lane & 31);
#pragma unroll
            for (int kk = 0; kk < 8; kk++) {
                if (kk < ksteps) {
                    v4i a = *(const v4i*)(tl + (size_t)arow * rowBytes + 16 * swz_chunk(arow, 2 * kk + half));
#pragma unroll
                    for (int g = 0; g < QG; g++)
                        acc.a[g] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bq[g][kk], acc.a[g], 0, 0, 0);
                }
            }
            return acc;
        };
        auto epi = [&](const Acc& acc, int rb, auto fullc) {
            // this lane's 16 train rows of the block; rows past nB exist only in the last tile,
            // tested against one per-lane limit (the row offsets stay compile-time constants)
            const int c = rb & 1;
            const int lim = nB - t * TR - 4 * half;
#pragma unroll
            for (int g = 0; g < QG; g++) {
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int row = rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                    uint32_t v = ((uint32_t)acc.a[g][r] << kShift) + ct[row];
                    if (!decltype(fullc)::value) v = (rb * 32 + (r & 3) + 8 * (r >> 2) < lim) ? v : 0u;
                    p2[g][c] = med3u(p1[g][c], p2[g][c], v);
                    p1[g][c] = umax(p1[g][c], v);
                }
            }
        };
        auto blocks = [&](auto fullc) {
            Acc accCur = mma(0);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int rb = 0; rb < TR / 32; rb++) {
                Acc accNext;
                if (rb + 1 < TR / 32) accNext = mma(rb + 1);
                epi(accCur, rb, fullc);
                // one scheduling region per block: at most two accumulator sets live (without the
                // barriers the compiler hoists all sixteen MFMAs: 194 VGPRs instead of 150)
                __builtin_amdgcn_sched_barrier(0);
                if (rb + 1 < TR / 32) accCur = accNext;
            }
        };
        if ((t + 1) * TR <= nB)
            blocks(std::true_type());
        else
            blocks(std::false_type());
        // merge the chains, then fold the tile's two best into the running (key, index) list:
        // earlier tiles hold lower indices, and top2_insert keeps them on equal keys
#pragma unroll
        for (int g = 0; g < QG; g++) {
            const uint32_t m1 = umax(p1[g][0], p1[g][1]);
            const uint32_t m2 = umax(umin(p1[g][0], p1[g][1]), umax(p2[g][0], p2[g][1]));
            if (m1)
                top2_insert((int)kBias - (int)(m1 >> kRB), t * TR + (int)kRowMask - (int)(m1 & kRowMask), b1[g], i1[g],
                            b2[g], i2[g]);
            if (m2)
                top2_insert((int)kBias - (int)(m2 >> kRB), t * TR + (int)kRowMask - (int)(m2 & kRowMask), b1[g], i1[g],
                            b2[g], i2[g]);
        }
        if (t + 1 < tEnd) store_tile(buf ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int g = 0; g < QG; g++) {
        // lanes l and l+32 hold the same query (different train rows): merge
        int c1 = __shfl_xor(b1[g], 32), j1 = __shfl_xor(i1[g], 32), c2 = __shfl_xor(b2[g], 32),
            j2 = __shfl_xor(i2[g], 32);
        top2_merge(b1[g], i1[g], b2[g], i2[g], c1, j1, c2, j2);
        const int qrow = q0 + 32 * g + (lane & 31);
        if (half == 0 && qrow < nA) {
            const int cq = BITS ? 0 : cqA[qrow];
            const size_t o = ((size_t)blockIdx.y * nA + qrow) * 2;
            idxOut[o] = i1[g];
            idxOut[o + 1] = i2[g];
            keyOut[o] = i1[g] >= 0 ? cq + b1[g] : INT_MAX;
            keyOut[o + 1] = i2[g] >= 0 ? cq + b2[g] : INT_MAX;
        }
    }
}

// ---------------- float rows, FLANN L2 order ----------------
// One query per thread, a[DIM] in registers.  The train rows are copied once into pairs,
// interleaved element by element, and read through scalar loads (every lane needs the same
// values), so one packed f32 instruction (v_pk_add / v_pk_mul, SGPR-pair operand) advances the
// distances to two rows: per lane the arithmetic is exactly FLANN's L2 order (groups of four,
// result += ((d0*d0 + d1*d1) + d2*d2) + d3*d3), just two rows at a time.  blockIdx.y selects a
// contiguous range of train rows (a part); the parts' top-2 lists are merged by knn2_f32_merge.
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ inline void top2_insert_f(float s, int j, float& b1, int& i1, float& b2, int& i2) {
    // the scan order's rule: strictly smaller replaces (ties keep the lower train index; NaN and
    // +inf never enter)
    const bool lt1 = s < b1, lt2 = s < b2;
    b2 = lt1 ? b1 : (lt2 ? s : b2);
    i2 = lt1 ? i1 : (lt2 ? j : i2);
    b1 = lt1 ? s : b1;
    i1 = lt1 ? j : i1;
}

// B in row pairs, interleaved element by element: P[(pr*DIM + d)*2 + k] = B[2pr + k][d] (zero
// past nB, nPairs rounded up to even so that the kernel may read pair pr + 1 unconditionally)
__global__ void f32_row_pairs_kernel(const float* __restrict__ B, int nB, int dim, int nPairs, float* __restrict__ P) {
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (size_t)nPairs * dim * 2) return;
    const int k = (int)(e & 1);
    const size_t pd = e >> 1;
    const int pr = (int)(pd / dim), d = (int)(pd - (size_t)pr * dim);
    const int j = 2 * pr + k;
    P[e] = j < nB ? B[(size_t)j * dim + d] : 0.f;
}

// (a.lo - b.lo, a.lo - b.hi) and (a.hi - b.lo, a.hi - b.hi) with b in an SGPR pair: one
// v_pk_add_f32 with src0's half broadcast by op_sel (the query row stays packed two elements
// per register pair)
__device__ inline f32x2 pk_sub_lo_s(f32x2 a, f32x2 b) {
    f32x2 d;
    asm("v_pk_add_f32 %0, %1, %2 op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d) : "v"(a), "s"(b));
    return d;
}
__device__ inline f32x2 pk_sub_hi_s(f32x2 a, f32x2 b) {
    f32x2 d;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d) : "v"(a), "s"(b));
    return d;
}

// the same scan with the train row pairs read through scalar loads (every lane of a wave needs
// the same train values): no LDS traffic, the SGPR pair is the packed instruction's operand
template <int DIM>
__global__ __launch_bounds__(256) void knn2_f32_sgpr_kernel(const float* __restrict__ A, int nA,
                                                            const float* __restrict__ P, int nB, int rowsPerPart,
                                                            int* __restrict__ idxOut, float* __restrict__ keyOut) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int jBeg = blockIdx.y * rowsPerPart;
    const int jEnd = min(nB, jBeg + rowsPerPart);
    f32x2 a[DIM / 2];
    {
        const float4* ap = reinterpret_cast<const float4*>(A + (size_t)min(q, nA - 1) * DIM);
#pragma unroll
        for (int k = 0; k < DIM / 4; k++) {
            const float4 v = ap[k];
            a[2 * k] = f32x2{v.x, v.y};
            a[2 * k + 1] = f32x2{v.z, v.w};
        }
    }
    float b1 = __builtin_inff(), b2 = __builtin_inff();
    int i1 = -1, i2 = -1;
    const float inf = __builtin_inff();
    for (int j = jBeg; j < jEnd; j += 4) {  // jBeg even: rows j..j+3 are pairs j/2, j/2 + 1
        const f32x2* b = reinterpret_cast<const f32x2*>(P) + (size_t)(j >> 1) * DIM;
        const f32x2* c = b + DIM;
        f32x2 res = {0.f, 0.f}, rec = {0.f, 0.f};
        // software pipeline: the scalar loads of group g + kAhead are issued before group g is used
        constexpr int kG = DIM / 4, kAhead = 3;
        f32x2 vb[kG][4], vc[kG][4];
#pragma unroll
        for (int g = 0; g < kAhead; g++)
#pragma unroll
            for (int t = 0; t < 4; t++) {
                vb[g][t] = b[4 * g + t];
                vc[g][t] = c[4 * g + t];
            }
#pragma unroll
        for (int g = 0; g < kG; g++) {
            if (g + kAhead < kG) {
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    vb[g + kAhead][t] = b[4 * (g + kAhead) + t];
                    vc[g + kAhead][t] = c[4 * (g + kAhead) + t];
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            const int i = 4 * g;
            const f32x2 d0 = pk_sub_lo_s(a[i / 2], vb[g][0]), d1 = pk_sub_hi_s(a[i / 2], vb[g][1]);
            const f32x2 d2 = pk_sub_lo_s(a[i / 2 + 1], vb[g][2]), d3 = pk_sub_hi_s(a[i / 2 + 1], vb[g][3]);
            const f32x2 e0 = pk_sub_lo_s(a[i / 2], vc[g][0]), e1 = pk_sub_hi_s(a[i / 2], vc[g][1]);
            const f32x2 e2 = pk_sub_lo_s(a[i / 2 + 1], vc[g][2]), e3 = pk_sub_hi_s(a[i / 2 + 1], vc[g][3]);
            res += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
            rec += e0 * e0 + e1 * e1 + e2 * e2 + e3 * e3;
        }
        top2_insert_f(res.x, j, b1, i1, b2, i2);
        top2_insert_f(j + 1 < jEnd ? res.y : inf, j + 1, b1, i1, b2, i2);
        top2_insert_f(j + 2 < jEnd ? rec.x : inf, j + 2, b1, i1, b2, i2);
        top2_insert_f(j + 3 < jEnd ? rec.y : inf, j + 3, b1, i1, b2, i2);
    }
    if (q < nA) {
        const size_t o = ((size_t)blockIdx.y * nA + q) * 2;
        idxOut[o] = i1;
        idxOut[o + 1] = i2;
        keyOut[o] = b1;
        keyOut[o + 1] = b2;
    }
}

// merges the parts' top-2 lists in part order (= train index order), with the scan's rule
__global__ void knn2_f32_merge(const int* __restrict__ pIdx, const float* __restrict__ pKey, int nA, int parts,
                               int* __restrict__ idxOut, float* __restrict__ keyOut) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nA) return;
    float b1 = __builtin_inff(), b2 = __builtin_inff();
    int i1 = -1, i2 = -1;
    for (int s = 0; s < parts; s++) {
        const size_t o = ((size_t)s * nA + q) * 2;
        int j0 = pIdx[o], j1 = pIdx[o + 1];
        float k0 = pKey[o], k1 = pKey[o + 1];
        if (j1 >= 0 && j1 < j0) {  // visit the part's two candidates in train index order
            const int tj = j0; j0 = j1; j1 = tj;
            const float tk = k0; k0 = k1; k1 = tk;
        }
        if (j0 >= 0) top2_insert_f(k0, j0, b1, i1, b2, i2);
        if (j1 >= 0) top2_insert_f(k1, j1, b1, i1, b2, i2);
    }
    idxOut[2 * q] = i1;
    idxOut[2 * q + 1] = i2;
    keyOut[2 * q] = b1;
    keyOut[2 * q + 1] = b2;
}

// generic dim: rows read from global memory (any dim, same FLANN order)
__global__ __launch_bounds__(256) void knn2_f32_generic_kernel(const float* __restrict__ A, int nA,
                                                               const float* __restrict__ B, int nB, int dim,
                                                               int* __restrict__ idxOut, float* __restrict__ keyOut) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nA) return;
    const float* a = A + (size_t)q * dim;
    float b1 = __builtin_inff(), b2 = __builtin_inff();
    int i1 = -1, i2 = -1;
    for (int j = 0; j < nB; j++) {
        const float* b = B + (size_t)j * dim;
        float result = 0.f;
        int i = 0;
        for (; i + 3 < dim; i += 4) {
            float d0 = a[i] - b[i], d1 = a[i + 1] - b[i + 1], d2 = a[i + 2] - b[i + 2], d3 = a[i + 3] - b[i + 3];
            result += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
        }
        for (; i < dim; i++) {
            float d0 = a[i] - b[i];
            result += d0 * d0;
        }
        if (result < b1) {
            b2 = b1;
            i2 = i1;
            b1 = result;
            i1 = j;
        } else if (result < b2) {
            b2 = result;
            i2 = j;
        }
    }
    idxOut[2 * q] = i1;
    idxOut[2 * q + 1] = i2;
    keyOut[2 * q] = b1;
    keyOut[2 * q + 1] = b2;
}

// ---------------- binary strings, Hamming ----------------
// One query per thread; the train rows are read through scalar loads (uniform across the wave:
// the words are SGPR operands of v_xor / v_bcnt, no LDS), over a train range (blockIdx.y, parts
// merged by knn2_int_merge); four rows per iteration
template <int NW>
__global__ __launch_bounds__(256) void knn2_bits_sgpr_kernel(const uint32_t* __restrict__ A, int nA,
                                                             const uint32_t* __restrict__ B, int nB, int rowsPerPart,
                                                             int* __restrict__ idxOut, int* __restrict__ keyOut) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int jBeg = blockIdx.y * rowsPerPart;
    const int jEnd = min(nB, jBeg + rowsPerPart);
    uint32_t a[NW];
    const uint32_t* ap = A + (size_t)min(q, nA - 1) * NW;
#pragma unroll
    for (int w = 0; w < NW; w++) a[w] = ap[w];
    int b1 = INT_MAX, b2 = INT_MAX, i1 = -1, i2 = -1;
    int j = jBeg;
    for (; j + 3 < jEnd; j += 4) {
        const uint32_t* r = B + (size_t)j * NW;
        int h[4] = {0, 0, 0, 0};
#pragma unroll
        for (int w = 0; w < NW; w++)
#pragma unroll
            for (int t = 0; t < 4; t++) h[t] += __popc(a[w] ^ r[t * NW + w]);
#pragma unroll
        for (int t = 0; t < 4; t++) top2_insert(h[t], j + t, b1, i1, b2, i2);
    }
    for (; j < jEnd; j++) {
        const uint32_t* r = B + (size_t)j * NW;
        int h = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) h += __popc(a[w] ^ r[w]);
        top2_insert(h, j, b1, i1, b2, i2);
    }
    if (q < nA) {
        const size_t o = ((size_t)blockIdx.y * nA + q) * 2;
        idxOut[o] = i1;
        idxOut[o + 1] = i2;
        keyOut[o] = b1;
        keyOut[o + 1] = b2;
    }
}

// merges the parts' top-2 lists (int keys) in part order with the scan's rule
__global__ void knn2_int_merge(const int* __restrict__ pIdx, const int* __restrict__ pKey, int nA, int parts,
                               int* __restrict__ idxOut, int* __restrict__ keyOut) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nA) return;
    int b1 = INT_MAX, b2 = INT_MAX, i1 = -1, i2 = -1;
    for (int s = 0; s < parts; s++) {
        const size_t o = ((size_t)s * nA + q) * 2;
        int j0 = pIdx[o], j1 = pIdx[o + 1];
        int k0 = pKey[o], k1 = pKey[o + 1];
        if (j1 >= 0 && j1 < j0) {  // visit the part's two candidates in train index order
            const int tj = j0; j0 = j1; j1 = tj;
            const int tk = k0; k0 = k1; k1 = tk;
        }
        if (j0 >= 0) top2_insert(k0, j0, b1, i1, b2, i2);
        if (j1 >= 0) top2_insert(k1, j1, b1, i1, b2, i2);
    }
    idxOut[2 * q] = i1;
    idxOut[2 * q + 1] = i2;
    keyOut[2 * q] = b1;
    keyOut[2 * q + 1] = b2;
}

__global__ void nndr_kernel(int type, const int* __restrict__ idx, const int* __restrict__ key,
                            const float* __restrict__ fkey, int nA, double eps, int queryOffset,
                            fm3d_dmatch* __restrict__ knnOut, fm3d_dmatch* __restrict__ cand, int* __restrict__ flag) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nA) return;
    const int i1 = idx[2 * q], i2 = idx[2 * q + 1];
    float d1, d2;
    if (type == FM3D_DESC_F32) {
        // FlannBasedMatcher::convertToDMatches: dist = sqrt(L2sqr) in float
        d1 = sqrtf(fkey[2 * q]);
        d2 = sqrtf(fkey[2 * q + 1]);
    } else if (type == FM3D_DESC_U8) {
        d1 = sqrtf((float)key[2 * q]);
        d2 = sqrtf((float)key[2 * q + 1]);
    } else {
        d1 = (float)key[2 * q];
        d2 = (float)key[2 * q + 1];
    }
    if (knnOut) {
        knnOut[2 * q] = fm3d_dmatch{q + queryOffset, i1, 0, d1};
        knnOut[2 * q + 1] = fm3d_dmatch{q + queryOffset, i2, 0, d2};
    }
    // descriptorsmatcher.cpp:121-128: size() >= 2 and distance0 <= epsilon * distance1 (double)
    const bool keep = (i1 >= 0 && i2 >= 0) && ((double)d1 <= eps * (double)d2);
    flag[q] = keep ? 1 : 0;
    cand[q] = fm3d_dmatch{q + queryOffset, i1, 0, d1};
}

// nndr_kernel with the parts' merge (knn2_int_merge's rule; int keys) and the stable compaction of the
// kept matches in one launch (fm3d_kernels.h LookBack): the pipeline's a1 without two launches and
// their round trips.  Block b's queries are b*256 .. b*256+255, b taken in launch order.
__global__ __launch_bounds__(256) void nndr_compact_kernel(int type, const int* __restrict__ idx,
                                                           const int* __restrict__ key, const float* __restrict__ fkey,
                                                           const int* __restrict__ pIdx, const int* __restrict__ pKey,
                                                           int parts, int nA, double eps, int queryOffset,
                                                           fm3d_dmatch* __restrict__ out, int* __restrict__ count,
                                                           LookBack lb) {
    __shared__ int sBid, sEx, sWave[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) sBid = lookback_block_id(lb);
    __syncthreads();
    const int bid = sBid;
    const int q = bid * 256 + tid;
    bool keep = false;
    fm3d_dmatch cand{};
    if (q < nA) {
        int i1, i2;
        float d1, d2;
        if (parts > 1) {
            int b1 = INT_MAX, b2 = INT_MAX;
            i1 = i2 = -1;
            auto merge_part = [&](int j0, int j1, int k0, int k1) {
                if (j1 >= 0 && j1 < j0) {  // visit the part's two candidates in train index order
                    const int tj = j0; j0 = j1; j1 = tj;
                    const int tk = k0; k0 = k1; k1 = tk;
                }
                if (j0 >= 0) top2_insert(k0, j0, b1, i1, b2, i2);
                if (j1 >= 0) top2_insert(k1, j1, b1, i1, b2, i2);
            };
            // the first 16 parts' lists loaded before any is merged (one round of load latency, not
            // one per part: 10.5 -> see DESIGN.md §3.2 at C2's 16 parts); knn2_u8_parts never makes
            // more, FM3D_I8_PARTS may
            int2 pj[16], pk[16];
#pragma unroll
            for (int s = 0; s < 16; s++) {
                if (s < parts) {
                    const size_t o = ((size_t)s * nA + q) * 2;
                    pj[s] = *(const int2*)(pIdx + o);
                    pk[s] = *(const int2*)(pKey + o);
                }
            }
#pragma unroll
            for (int s = 0; s < 16; s++)
                if (s < parts) merge_part(pj[s].x, pj[s].y, pk[s].x, pk[s].y);
            for (int s = 16; s < parts; s++) {
                const size_t o = ((size_t)s * nA + q) * 2;
                merge_part(pIdx[o], pIdx[o + 1], pKey[o], pKey[o + 1]);
            }
            if (type == FM3D_DESC_U8) {
                d1 = sqrtf((float)b1);
                d2 = sqrtf((float)b2);
            } else {
                d1 = (float)b1;
                d2 = (float)b2;
            }
        } else {
            i1 = idx[2 * q];
            i2 = idx[2 * q + 1];
            if (type == FM3D_DESC_F32) {
                d1 = sqrtf(fkey[2 * q]);
                d2 = sqrtf(fkey[2 * q + 1]);
            } else if (type == FM3D_DESC_U8) {
                d1 = sqrtf((float)key[2 * q]);
                d2 = sqrtf((float)key[2 * q + 1]);
            } else {
                d1 = (float)key[2 * q];
                d2 = (float)key[2 * q + 1];
            }
        }
        // descriptorsmatcher.cpp:121-128: size() >= 2 and distance0 <= epsilon * distance1 (double)
        keep = (i1 >= 0 && i2 >= 0) && ((double)d1 <= eps * (double)d2);
        cand = fm3d_dmatch{q + queryOffset, i1, 0, d1};
    }
    const unsigned long long bal = __ballot(keep);
    if (lane == 0) sWave[wave] = __popcll(bal);
    __syncthreads();
    if (wave == 0) {
        const int ex = lookback_exclusive(lb.st, lb.epoch, bid, sWave[0] + sWave[1] + sWave[2] + sWave[3]);
        if (lane == 0) sEx = ex;
    }
    __syncthreads();
    int o = sEx + __popcll(bal & ((1ull << lane) - 1));
    for (int w = 0; w < wave; w++) o += sWave[w];
    if (keep) out[o] = cand;
    if (tid == 0 && bid == (int)gridDim.x - 1) *count = sEx + sWave[0] + sWave[1] + sWave[2] + sWave[3];
}

// ---------------- float rows: a bf16 MFMA prefilter, then the exact FLANN-order distances ----------------
// s'_j = |b_j|^2 - 2 a_hi . b_hi,j (a_hi, b_hi = the rows rounded to bf16; the dot products on
// v_mfma_f32_32x32x16_bf16, |b_j|^2 in fp32) ranks train row j for query a up to
//   |s'_j - s_j| <= eps_q = 0.0079 |a| Bmax + 1e-5 Bmax^2        (s_j = |a - b_j|^2 - |a|^2)
// (bf16 rounding 2^-9 per element, an exact bf16 product and <= 127 fp32 roundings per dot, the
// fp32 norm), and FLANN's float L2 is within phi_q = 2e-5 (|a| + Bmax)^2 of the true distance
// (dim <= 128).  So every member of the exact top-2 has s'_j <= s'_(2) + 2 eps_q + 2 phi_q: pass 1
// finds s'_(2), pass 2 lists the rows under that bound, pass 3 computes their exact FLANN-order
// distances and keeps the (distance, index) top-2 -- the same two rows and keys the full exact scan
// returns.  A query with more than kCandMax such rows, or a non-finite norm, is rescanned exactly.
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
constexpr int kCandMax = 32;
constexpr int kCandMax2 = 128;  // the fused pass: a lane's running records (~2 ln N) come on top

__device__ inline uint32_t bf16_rne(float x) {
    const uint32_t u = __float_as_uint(x);
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// rows (dim 64 / 128) -> bf16 rows, 8 elements (16 bytes) per thread; |row|^2 in fp32; the largest
// train |b|^2 into *bmax (as ordered bits: non-negative floats compare as ints)
__global__ void f32_bf16_rows_kernel(const float* __restrict__ A, int nA, const float* __restrict__ B, int nB, int dim,
                                     uint16_t* __restrict__ outA, uint16_t* __restrict__ outB, float* __restrict__ nA2,
                                     float* __restrict__ nB2, unsigned* __restrict__ bmax) {
    const int cpr = dim / 8;  // 8 or 16 lanes per row
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long r = t / cpr;
    const int k = (int)(t - r * cpr);
    const bool isA = r < nA;
    const long long rr = isA ? r : r - nA;
    float s = 0.f;
    if (r < (long long)nA + nB) {
        const float4* x = (const float4*)((isA ? A : B) + rr * dim + 8 * k);
        const float4 u = x[0], v = x[1];
        const float e[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
        v4i o;
#pragma unroll
        for (int w = 0; w < 4; w++) o[w] = (int)(bf16_rne(e[2 * w]) | (bf16_rne(e[2 * w + 1]) << 16));
        *(v4i*)((isA ? outA : outB) + rr * dim + 8 * k) = o;
#pragma unroll
        for (int w = 0; w < 8; w++) s += e[w] * e[w];
    }
    for (int o = 1; o < cpr; o <<= 1) s += __shfl_xor(s, o);
    if (k == 0 && r < (long long)nA + nB) {
        if (isA) {
            nA2[rr] = s;
        } else {
            nB2[rr] = s;
            atomicMax(bmax, (s == s && s <= 3.4e38f) ? __float_as_uint(s) : 0x7f800000u);  // non-finite: +inf
        }
    }
}

// MODE 0: per (part, query) the two smallest s'; MODE 1: the rows with s' <= thr[q] appended to the
// query's candidate list.  The tiling is knn2_i8_kernel's (128 queries x 128-row LDS tiles, the
// query row as the MFMA's B operand; a bf16 k-step is the same 32 bytes as an int8 one).
template <int KS, int MODE>
__global__ __launch_bounds__(kThreads) void knn2_bf16_kernel(const uint16_t* __restrict__ A, int nA,
                                                             const uint16_t* __restrict__ B, int nB,
                                                             const float* __restrict__ nb2, int tilesPerPart,
                                                             const float* __restrict__ thr, float* __restrict__ keyOut,
                                                             int* __restrict__ cnt, int* __restrict__ cand,
                                                             float* __restrict__ candKey) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int rowBytes = 32 * KS, tileBytes = kT * rowBytes, chunksPerRow = rowBytes / 16;
    unsigned char* tiles = smem;                           // 2 x tileBytes
    float* ctl = (float*)(smem + 2 * (size_t)tileBytes);    // 2 x kT |b|^2
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int qrow = blockIdx.x * kQ + wave * 32 + (lane & 31);
    const int half = lane >> 5;
    v4i bq[KS];
#pragma unroll
    for (int kk = 0; kk < KS; kk++) {
        v4i v = {0, 0, 0, 0};
        if (qrow < nA) v = *(const v4i*)((const unsigned char*)A + (size_t)qrow * rowBytes + 32 * kk + 16 * half);
        bq[kk] = v;
    }
    const float inf = __builtin_inff();
    // MODE 1: the bound; MODE 2: the margin added to the running second-best
    const float tq = (MODE != 0 && qrow < nA) ? thr[qrow] : -inf;
    float p1 = inf, p2 = inf;
    const int tBeg = blockIdx.y * tilesPerPart;
    const int tEnd = min((nB + kT - 1) / kT, tBeg + tilesPerPart);
    constexpr int kPre = (kT * chunksPerRow + kThreads - 1) / kThreads;
    constexpr int total = kT * chunksPerRow;
    v4i pre[kPre];
    float preCt = inf;
    auto load_tile = [&](int t) {
#pragma unroll
        for (int i = 0; i < kPre; i++) {
            const int c = tid + i * kThreads;
            v4i v = {0, 0, 0, 0};
            if (c < total) {
                const int row = c / chunksPerRow, ch = c - row * chunksPerRow;
                const int j = t * kT + row;
                if (j < nB) v = *(const v4i*)((const unsigned char*)B + (size_t)j * rowBytes + 16 * ch);
            }
            pre[i] = v;
        }
        if (tid < kT) {
            const int j = t * kT + tid;
            preCt = (j < nB) ? nb2[j] : inf;  // rows past nB: +inf never ranks
        }
    };
    auto store_tile = [&](int buf) {
        unsigned char* dst = tiles + (size_t)buf * tileBytes;
#pragma unroll
        for (int i = 0; i < kPre; i++) {
            const int c = tid + i * kThreads;
            if (c < total) {
                const int row = c / chunksPerRow, ch = c - row * chunksPerRow;
                *(v4i*)(dst + (size_t)row * rowBytes + 16 * swz_chunk(row, ch)) = pre[i];
            }
        }
        if (tid < kT) ctl[buf * kT + tid] = preCt;
    };
    if (tBeg < tEnd) {
        load_tile(tBeg);
        store_tile(0);
    }
    __syncthreads();
    for (int t = tBeg; t < tEnd; t++) {
        const int buf = (t - tBeg) & 1;
        if (t + 1 < tEnd) load_tile(t + 1);
        const unsigned char* tl = tiles + (size_t)buf * tileBytes;
        const float* ct = ctl + buf * kT;
        auto mma = [&](int rb) {
            v16f acc = {0};
            const int arow = rb * 32 + (lane & 31);
#pragma unroll
            for (int kk = 0; kk < KS; kk++) {
                const v4i a = *(const v4i*)(tl + (size_t)arow * rowBytes + 16 * swz_chunk(arow, 2 * kk + half));
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, bq[kk]),
                                                              acc, 0, 0, 0);
            }
            return acc;
        };
        v16f accCur = mma(0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rb = 0; rb < kT / 32; rb++) {
            v16f accNext;
            if (rb + 1 < kT / 32) accNext = mma(rb + 1);
            unsigned hits = 0;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int row = rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                const float v = fmaf(-2.f, accCur[r], ct[row]);
                if (MODE != 1) {
                    p2 = __builtin_amdgcn_fmed3f(p1, p2, v);
                    p1 = fminf(p1, v);
                }
                if (MODE == 1) hits |= (v <= tq ? 1u : 0u) << r;
                // MODE 2: under this lane's running second-best + the margin (>= the final bound)
                if (MODE == 2) hits |= (v <= p2 + tq ? 1u : 0u) << r;
            }
            if (MODE != 0 && hits) {
                do {
                    const int r = __builtin_ctz(hits);
                    hits &= hits - 1;
                    const int j = t * kT + rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                    const int slot = atomicAdd(&cnt[qrow], 1);
                    if (MODE == 1 && slot < kCandMax) cand[(size_t)qrow * kCandMax + slot] = j;
                    if (MODE == 2 && slot < kCandMax2) {
                        cand[(size_t)qrow * kCandMax2 + slot] = j;
                        candKey[(size_t)qrow * kCandMax2 + slot] = fmaf(-2.f, accCur[r], ct[rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * half]);
                    }
                } while (hits);
            }
            __builtin_amdgcn_sched_barrier(0);
            if (rb + 1 < kT / 32) accCur = accNext;
        }
        if (t + 1 < tEnd) store_tile(buf ^ 1);
        __syncthreads();
    }
    if (MODE != 1) {
        // lanes l and l + 32 hold the same query (the other 16 rows of every block)
        const float q1 = __shfl_xor(p1, 32), q2 = __shfl_xor(p2, 32);
        const float n1 = fminf(p1, q1), n2 = fminf(fmaxf(p1, q1), fminf(p2, q2));
        if (half == 0 && qrow < nA) {
            const size_t o = ((size_t)blockIdx.y * nA + qrow) * 2;
            keyOut[o] = n1;
            keyOut[o + 1] = n2;
        }
    }
}

// the bound thr[q] = s'_(2) over all parts + 2 eps_q + 2 phi_q (+ slack), rounded up; cnt[q] = 0.
// A non-finite norm or bound sends the query to the exact rescan (thr = -inf, cnt = kCandMax + 1).
__global__ void knn2_bf16_bound_kernel(const float* __restrict__ partKey, int nA, int parts,
                                       const float* __restrict__ nA2, const unsigned* __restrict__ bmax,
                                       float* __restrict__ thr, int* __restrict__ cnt) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nA) return;
    float p1 = __builtin_inff(), p2 = __builtin_inff();
    for (int s = 0; s < parts; s++) {
        const size_t o = ((size_t)s * nA + q) * 2;
        const float c1 = partKey[o], c2 = partKey[o + 1];
        p2 = fminf(fmaxf(p1, c1), fminf(p2, c2));
        p1 = fminf(p1, c1);
    }
    const double a = sqrt((double)nA2[q]), bm = sqrt((double)__uint_as_float(*bmax));
    const double eps = 0.0079 * a * bm + 1e-5 * bm * bm, phi = 2e-5 * (a + bm) * (a + bm);
    const double t = (double)p2 + 2 * eps + 2 * phi + 1e-6 * (a + bm) * (a + bm);
    // (rows of norm below 1e-10 are rescanned: the bound does not cover the MFMA's denormal handling)
    const bool ok = t == t && t < 1e37 && a < 1e18 && a + bm > 1e-10;
    float t32 = (float)t;
    if ((double)t32 < t) t32 = nextafterf(t32, __builtin_inff());  // rounded up
    thr[q] = ok ? t32 : -__builtin_inff();
    cnt[q] = ok ? 0 : kCandMax + 1;
}

// FLANN L2<float> (flann/dist.h): groups of four, result += d0^2 + d1^2 + d2^2 + d3^2, then the tail
__device__ inline float flann_l2(const float* __restrict__ a, const float* __restrict__ b, int dim) {
    float result = 0.f;
    int i = 0;
    for (; i + 3 < dim; i += 4) {
        const float d0 = a[i] - b[i], d1 = a[i + 1] - b[i + 1], d2 = a[i + 2] - b[i + 2], d3 = a[i + 3] - b[i + 3];
        result += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
    }
    for (; i < dim; i++) {
        const float d0 = a[i] - b[i];
        result += d0 * d0;
    }
    return result;
}

__device__ inline bool lex_lt_f(float a, int ia, float b, int ib) { return a < b || (a == b && ia < ib); }

// the candidates' exact distances, (distance, index) top-2; overflowing queries into the rescan list
__global__ void knn2_f32_recheck_kernel(const float* __restrict__ A, int nA, const float* __restrict__ B, int dim,
                                        const int* __restrict__ cnt, const int* __restrict__ cand,
                                        int* __restrict__ idxOut, float* __restrict__ keyOut,
                                        int* __restrict__ resc, int* __restrict__ nResc) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nA) return;
    const int n = cnt[q];
    if (n > kCandMax) {
        resc[atomicAdd(nResc, 1)] = q;
        return;
    }
    const float* a = A + (size_t)q * dim;
    float b1 = __builtin_inff(), b2 = __builtin_inff();
    int i1 = -1, i2 = -1;
    for (int c = 0; c < n; c++) {
        const int j = cand[(size_t)q * kCandMax + c];
        const float d = flann_l2(a, B + (size_t)j * dim, dim);
        if (!(d < __builtin_inff())) continue;  // NaN / +inf never enter (the scan's rule)
        if (lex_lt_f(d, j, b1, i1 < 0 ? INT_MAX : i1)) {
            b2 = b1;
            i2 = i1;
            b1 = d;
            i1 = j;
        } else if (lex_lt_f(d, j, b2, i2 < 0 ? INT_MAX : i2)) {
            b2 = d;
            i2 = j;
        }
    }
    idxOut[2 * q] = i1;
    idxOut[2 * q + 1] = i2;
    keyOut[2 * q] = b1;
    keyOut[2 * q + 1] = b2;
}

// the fused pass's per-query margin 2 eps_q + 2 phi_q + slack (rounded up); cnt[q] = 0, or the
// rescan mark (margin -inf) for a non-finite norm
__global__ void knn2_bf16_margin_kernel(const float* __restrict__ nA2, int nA, const unsigned* __restrict__ bmax,
                                        float* __restrict__ margin, int* __restrict__ cnt) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nA) return;
    const double a = sqrt((double)nA2[q]), bm = sqrt((double)__uint_as_float(*bmax));
    const double m = 2 * (0.0079 * a * bm + 1e-5 * bm * bm) + 2 * 2e-5 * (a + bm) * (a + bm) + 1e-6 * (a + bm) * (a + bm);
    const bool ok = m == m && m < 1e37 && a < 1e18 && a + bm > 1e-10;
    float m32 = (float)m;
    if ((double)m32 < m) m32 = nextafterf(m32, __builtin_inff());
    margin[q] = ok ? m32 : -__builtin_inff();
    cnt[q] = ok ? 0 : kCandMax2 + 1;
}

// the fused pass's candidates: those under the final bound s'_(2) + margin get their exact
// FLANN-order distances; (distance, index) top-2; overflowing queries into the rescan list
__global__ void knn2_f32_recheck2_kernel(const float* __restrict__ A, int nA, const float* __restrict__ B, int dim,
                                         const float* __restrict__ partKey, int parts, const float* __restrict__ margin,
                                         const int* __restrict__ cnt, const int* __restrict__ cand,
                                         const float* __restrict__ candKey, int* __restrict__ idxOut,
                                         float* __restrict__ keyOut, int* __restrict__ resc, int* __restrict__ nResc) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nA) return;
    const int n = cnt[q];
    if (n > kCandMax2) {
        resc[atomicAdd(nResc, 1)] = q;
        return;
    }
    float p1 = __builtin_inff(), p2 = __builtin_inff();
    for (int s = 0; s < parts; s++) {
        const size_t o = ((size_t)s * nA + q) * 2;
        const float c1 = partKey[o], c2 = partKey[o + 1];
        p2 = fminf(fmaxf(p1, c1), fminf(p2, c2));
        p1 = fminf(p1, c1);
    }
    const float T = p2 + margin[q];  // the fp32 add rounds: the candidates were emitted under larger bounds
    const float* a = A + (size_t)q * dim;
    float b1 = __builtin_inff(), b2 = __builtin_inff();
    int i1 = -1, i2 = -1;
    for (int c = 0; c < n; c++) {
        if (!(candKey[(size_t)q * kCandMax2 + c] <= nextafterf(T, __builtin_inff()))) continue;
        const int j = cand[(size_t)q * kCandMax2 + c];
        const float d = flann_l2(a, B + (size_t)j * dim, dim);
        if (!(d < __builtin_inff())) continue;
        if (lex_lt_f(d, j, b1, i1 < 0 ? INT_MAX : i1)) {
            b2 = b1;
            i2 = i1;
            b1 = d;
            i1 = j;
        } else if (lex_lt_f(d, j, b2, i2 < 0 ? INT_MAX : i2)) {
            b2 = d;
            i2 = j;
        }
    }
    idxOut[2 * q] = i1;
    idxOut[2 * q + 1] = i2;
    keyOut[2 * q] = b1;
    keyOut[2 * q + 1] = b2;
}

// the exact scan for the listed queries: a wave per query, lane l takes rows l, l + 64, ... (in
// increasing order, the scan's rule per lane), then the lanes' lists merge lexicographically
__global__ __launch_bounds__(256) void knn2_f32_rescan_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                              int nB, int dim, const int* __restrict__ resc,
                                                              const int* __restrict__ nResc, int* __restrict__ idxOut,
                                                              float* __restrict__ keyOut) {
    const int lane = threadIdx.x & 63;
    const int n = *nResc;
    for (int w = blockIdx.x * 4 + (threadIdx.x >> 6); w < n; w += gridDim.x * 4) {
        const int q = resc[w];
        const float* a = A + (size_t)q * dim;
        float b1 = __builtin_inff(), b2 = __builtin_inff();
        int i1 = -1, i2 = -1;
        for (int j = lane; j < nB; j += 64) top2_insert_f(flann_l2(a, B + (size_t)j * dim, dim), j, b1, i1, b2, i2);
        for (int o = 1; o < 64; o <<= 1) {
            const float c1 = __shfl_xor(b1, o), c2 = __shfl_xor(b2, o);
            const int j1 = __shfl_xor(i1, o), j2 = __shfl_xor(i2, o);
            // merge (b1, i1, b2, i2) with (c1, j1, c2, j2) lexicographically (-1 = none, sorts last)
            const int k1 = i1 < 0 ? INT_MAX : i1, k2 = i2 < 0 ? INT_MAX : i2;
            const int l1 = j1 < 0 ? INT_MAX : j1, l2 = j2 < 0 ? INT_MAX : j2;
            float r1, r2;
            int s1, s2;
            if (lex_lt_f(b1, k1, c1, l1)) {
                r1 = b1, s1 = k1;
                if (lex_lt_f(b2, k2, c1, l1)) r2 = b2, s2 = k2; else r2 = c1, s2 = l1;
            } else {
                r1 = c1, s1 = l1;
                if (lex_lt_f(b1, k1, c2, l2)) r2 = b1, s2 = k1; else r2 = c2, s2 = l2;
            }
            b1 = r1, i1 = s1 == INT_MAX ? -1 : s1;
            b2 = r2, i2 = s2 == INT_MAX ? -1 : s2;
        }
        if (lane == 0) {
            idxOut[2 * q] = i1;
            idxOut[2 * q + 1] = i2;
            keyOut[2 * q] = b1;
            keyOut[2 * q + 1] = b2;
        }
    }
}

// Float rows handed over as the reference's cv::Mat of SIFT descriptors (descriptorsmatcher.cpp:114-117)
// that hold integers in [0, 255] (OpenCV's SIFT saturates to uchar before the float conversion): each
// thread packs 4 bytes of a u8 row padded to dimPad (pad value 128) for the int8-MFMA kernel, both
// sides in one launch, and *notU8 becomes 1 when any element is not such an integer (NaN included),
// so the host keeps the float kernels.  (Until round 6 the host scanned and converted the rows on the
// submitting thread.)
__global__ __launch_bounds__(256) void f32_pack_u8_kernel(const float* __restrict__ A, unsigned nA,
                                                          const float* __restrict__ B, unsigned nB, int dim,
                                                          int dimPad, uint8_t* __restrict__ Au,
                                                          uint8_t* __restrict__ Bu, int* __restrict__ notU8) {
    const unsigned q = (unsigned)dimPad >> 2;  // 4-byte groups per padded row
    const unsigned gA = nA * q, total = gA + nB * q;
    const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
    bool bad = false;
    if (t < total) {
        const bool isA = t < gA;
        const unsigned g = isA ? t : t - gA;
        const unsigned row = g / q;
        const int c0 = (int)(g - row * q) * 4;
        const float* src = (isA ? A : B) + (size_t)row * dim;
        float v[4];
        if ((dim & 3) == 0 && c0 + 4 <= dim) {
            const float4 f = *(const float4*)(src + c0);
            v[0] = f.x, v[1] = f.y, v[2] = f.z, v[3] = f.w;
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = c0 + k < dim ? src[c0 + k] : 128.f;
        }
        uint32_t packed = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const bool ok = v[k] >= 0.f && v[k] <= 255.f && v[k] == floorf(v[k]);
            bad |= !ok;
            packed |= (ok ? (uint32_t)v[k] : 0u) << (8 * k);
        }
        ((uint32_t*)(isA ? Au : Bu))[g] = packed;
    }
    const unsigned long long m = __ballot(bad);
    if (m && (int)(threadIdx.x & 63) == __ffsll((long long)m) - 1) atomicOr(notU8, 1);
}

}  // namespace

void launch_rowconst_u8(const uint8_t* A, int nA, const uint8_t* B, int nB, int dimPad, int* cq, int* ctp,
                        hipStream_t s) {
    const size_t threads = (size_t)(nA + nB) * (dimPad / 16);
    if (threads == 0) return;
    const int rowBits = knn2_i8_tile_rows(dimPad, 0) == 256 ? 8 : 7;
    rowconst_u8_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(A, nA, B, nB, dimPad, cq, ctp, rowBits);
}

void launch_f32_pack_u8(const float* A, int nA, const float* B, int nB, int dim, int dimPad, uint8_t* Au,
                        uint8_t* Bu, int* notU8, hipStream_t s) {
    const size_t groups = ((size_t)nA + nB) * (dimPad / 4);
    if (groups == 0) return;
    f32_pack_u8_kernel<<<(unsigned)((groups + 255) / 256), 256, 0, s>>>(A, (unsigned)nA, B, (unsigned)nB, dim, dimPad,
                                                                       Au, Bu, notU8);
}

void launch_unpack_bits(const uint8_t* A, int nA, const uint8_t* B, int nB, uint8_t* outA, uint8_t* outB, int* ctp,
                        hipStream_t s) {
    if (nA + nB <= 0) return;
    unpack_bits_kernel<<<((nA + nB) * 8 + 255) / 256, 256, 0, s>>>((const uint32_t*)A, nA, (const uint32_t*)B, nB,
                                                                (int8_t*)outA, (int8_t*)outB, ctp);
}

void launch_knn2_i8(const uint8_t* A, int nA, const uint8_t* B, int nB, int dimPad, int bits, const int* cqA,
                    const int* ctB, int parts, int* partIdx, int* partKey, int* idx, int* key, hipStream_t s,
                    bool deferMerge) {
    if (nA <= 0) return;
    const int TRv = knn2_i8_tile_rows(dimPad, bits);
    size_t lds = 2 * (size_t)TRv * dimPad + 2 * TRv * sizeof(int);
    const int nTiles = (nB + TRv - 1) / TRv;
    const int tilesPerPart = parts > 1 ? (nTiles + parts - 1) / parts : (nTiles > 0 ? nTiles : 1);
    int* oi = parts > 1 ? partIdx : idx;
    int* ok = parts > 1 ? partKey : key;
    auto go = [&](auto kernel, int qg) {
        if (lds > 65536)
            (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        const dim3 g((nA + kQ * qg - 1) / (kQ * qg), parts);
        kernel<<<g, kThreads, lds, s>>>(A, nA, B, nB, dimPad, cqA, ctB, tilesPerPart, oi, ok);
    };
    if (bits)
        go(knn2_i8_kernel<8, true, 1>, 1);  // 32-byte binary rows unpacked to 256 int8
    else if (dimPad == 128)
        go(knn2_i8_kernel<4, false, kQG128, kTR128>, kQG128);
    else if (dimPad == 256)
        go(knn2_i8_kernel<8, false, 1>, 1);
    else
        go(knn2_i8_kernel<0, false, 1>, 1);
    if (parts > 1 && !deferMerge) knn2_int_merge<<<(nA + 255) / 256, 256, 0, s>>>(partIdx, partKey, nA, parts, idx, key);
}

size_t knn2_f32_mfma_bytes(int nA, int nB, int dim, int parts) {
    // bf16 rows, norms, bound, candidate lists (+ keys), part keys, rescan list (+ alignment slack)
    return (size_t)(nA + nB) * dim * 2 + (size_t)(nA + nB) * 4 + 64 + (size_t)nA * 4 * 3 + (size_t)nA * kCandMax2 * 8 +
           (size_t)parts * nA * 2 * 4 + (size_t)nA * 4 + 16 * 256;
}



// the bf16 prefilter kernel: parts only for query sets that leave CUs idle.  The int8 kernel's part
// model for large sets (the last partial round of blocks) made the fused pass slower here (100k x
// 100k SURF-128: 11.3 / 12.0 -> 17.7 / 17.8 ms, tools/r05_f32_parts_ab.sh): a part's running bound
// starts loose again, so more rows enter the candidate lists
int knn2_f32_mfma_parts(int nA, int nB, int nCU) { return knn2_u8_parts(nA, nB, nCU, 0, 0); }

void launch_knn2_f32_mfma(const float* A, int nA, const float* B, int nB, int dim, int parts, bool fused, void* work,
                          int* idx, float* key, hipStream_t s) {
    if (nA <= 0) return;
    char* w = (char*)work;
    auto take = [&](size_t bytes) {
        char* p = w;
        w += (bytes + 255) & ~(size_t)255;
        return p;
    };
    uint16_t* a16 = (uint16_t*)take((size_t)nA * dim * 2);
    uint16_t* b16 = (uint16_t*)take((size_t)nB * dim * 2);
    float* nA2 = (float*)take((size_t)nA * 4);
    float* nB2 = (float*)take((size_t)nB * 4);
    unsigned* bmax = (unsigned*)take(64);
    float* thr = (float*)take((size_t)nA * 4);
    int* cnt = (int*)take((size_t)nA * 4);
    int* cand = (int*)take((size_t)nA * kCandMax2 * 4);
    float* candKey = (float*)take((size_t)nA * kCandMax2 * 4);
    float* partKey = (float*)take((size_t)parts * nA * 2 * 4);
    int* resc = (int*)take((size_t)nA * 4);
    int* nResc = (int*)take(64);
    (void)hipMemsetAsync(bmax, 0, 4, s);
    (void)hipMemsetAsync(nResc, 0, 4, s);
    const long long thr8 = (long long)(nA + nB) * (dim / 8);
    f32_bf16_rows_kernel<<<(unsigned)((thr8 + 255) / 256), 256, 0, s>>>(A, nA, B, nB, dim, a16, b16, nA2, nB2, bmax);
    const int KS = dim / 16;
    const size_t lds = 2 * (size_t)kT * 32 * KS + 2 * kT * sizeof(float);
    const int nTiles = (nB + kT - 1) / kT;
    const int tilesPerPart = parts > 1 ? (nTiles + parts - 1) / parts : (nTiles > 0 ? nTiles : 1);
    const dim3 g((nA + kQ - 1) / kQ, parts);
    auto go = [&](auto k0, auto k1, auto k2) {
        if (lds > 65536) {
            (void)hipFuncSetAttribute((const void*)k0, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            (void)hipFuncSetAttribute((const void*)k1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            (void)hipFuncSetAttribute((const void*)k2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        }
        if (fused) {
            knn2_bf16_margin_kernel<<<(nA + 255) / 256, 256, 0, s>>>(nA2, nA, bmax, thr, cnt);
            k2<<<g, kThreads, lds, s>>>(a16, nA, b16, nB, nB2, tilesPerPart, thr, partKey, cnt, cand, candKey);
            knn2_f32_recheck2_kernel<<<(nA + 255) / 256, 256, 0, s>>>(A, nA, B, dim, partKey, parts, thr, cnt, cand,
                                                                      candKey, idx, key, resc, nResc);
        } else {
            k0<<<g, kThreads, lds, s>>>(a16, nA, b16, nB, nB2, tilesPerPart, nullptr, partKey, nullptr, nullptr,
                                        nullptr);
            knn2_bf16_bound_kernel<<<(nA + 255) / 256, 256, 0, s>>>(partKey, nA, parts, nA2, bmax, thr, cnt);
            k1<<<g, kThreads, lds, s>>>(a16, nA, b16, nB, nB2, tilesPerPart, thr, nullptr, cnt, cand, nullptr);
            knn2_f32_recheck_kernel<<<(nA + 255) / 256, 256, 0, s>>>(A, nA, B, dim, cnt, cand, idx, key, resc, nResc);
        }
    };
    if (KS == 8)
        go(knn2_bf16_kernel<8, 0>, knn2_bf16_kernel<8, 1>, knn2_bf16_kernel<8, 2>);
    else
        go(knn2_bf16_kernel<4, 0>, knn2_bf16_kernel<4, 1>, knn2_bf16_kernel<4, 2>);
}

int* knn2_f32_mfma_rescan_count(void* work, int nA, int nB, int dim, int parts) {
    // the last slot of launch_knn2_f32_mfma's layout
    size_t o = 0;
    auto take = [&](size_t bytes) { o += (bytes + 255) & ~(size_t)255; };
    take((size_t)nA * dim * 2);
    take((size_t)nB * dim * 2);
    take((size_t)nA * 4);
    take((size_t)nB * 4);
    take(64);
    take((size_t)nA * 4);
    take((size_t)nA * 4);
    take((size_t)nA * kCandMax2 * 4);
    take((size_t)nA * kCandMax2 * 4);
    take((size_t)parts * nA * 2 * 4);
    take((size_t)nA * 4);
    return (int*)((char*)work + o);
}

void launch_knn2_f32_mfma_rescan(const float* A, const float* B, int nB, int dim, void* work, int nA, int parts,
                                 int nResc, int* idx, float* key, hipStream_t s) {
    if (nResc <= 0) return;
    int* nR = knn2_f32_mfma_rescan_count(work, nA, nB, dim, parts);
    const int* resc = nR - ((((size_t)nA * 4) + 255) & ~(size_t)255) / sizeof(int);
    const int grid = (nResc + 3) / 4 < 1024 ? (nResc + 3) / 4 : 1024;
    knn2_f32_rescan_kernel<<<grid, 256, 0, s>>>(A, B, nB, dim, resc, nR, idx, key);
}

int knn2_i8_queries_per_block(int dimPad, int bits) { return (!bits && dimPad == 128 ? kQG128 : 1) * kQ; }
int knn2_i8_tile_rows(int dimPad, int bits) { return !bits && dimPad == 128 ? kTR128 : kT; }

int knn2_u8_parts(int nA, int nB, int nCU, int qPerBlock, int tileRows) {
    // Fewer query blocks than CUs: split the train tiles, aiming at four blocks per CU, each part
    // keeping >= 4 tiles: at 10k x 10k (79 query blocks) 16 parts take the u8 kernel 63 -> 29 us and
    // the bits kernel 56 -> 43 us (rocprofv3, MI355X).
    // More query blocks than CUs (qPerBlock > 0: the kernel's queries per workgroup): a CU's time
    // is its share of blocks times their length, so a last partial round of blocks costs almost a
    // whole one (100k x 100k at 128 queries: 782 blocks on 256 CUs).  Pick the part count p <= 16
    // (>= 4 tiles per part) minimising ceil(blocks * p / CUs) * ceil(tiles / p).  At 100k x 100k
    // (u8, 256 queries per block) p = 4, 8, 16 measured 2.01, 1.88, 1.80 ms against the model's
    // 1.12 : 1.04 : 1 (tools/knn_parts_sweep.py under rocprofv3; p = 1 at 128 queries: 2.87 ms).
    // FM3D_I8_PARTS overrides the part count (a tuning-only knob, read on every call so A/B runs in
    // one process see changes); it is clamped to [1, tiles].
    const char* e = getenv("FM3D_I8_PARTS");
    const int forced = e ? atoi(e) : 0;
    const int qb = qPerBlock > 0 ? qPerBlock : kQ;
    const int tr = tileRows > 0 ? tileRows : kT;
    const int nBlk = (nA + qb - 1) / qb;
    const int nTiles = (nB + tr - 1) / tr;
    if (nBlk <= 0 || nCU <= 0) return 1;
    if (forced > 0) return forced < (nTiles > 1 ? nTiles : 1) ? forced : (nTiles > 1 ? nTiles : 1);
    if (nBlk >= nCU) {
        if (qPerBlock <= 0) return 1;
        int best = 1;
        long long bestCost = 0;
        for (int p = 1; p <= 16; p++) {
            if (p > 1 && nTiles / p < 4) break;
            const long long cost = (((long long)nBlk * p + nCU - 1) / nCU) * ((nTiles + p - 1) / p);
            if (p == 1 || cost < bestCost) {
                best = p;
                bestCost = cost;
            }
        }
        return best;
    }
    int p = (4 * nCU + nBlk - 1) / nBlk;
    if (p > 16) p = 16;
    while (p > 1 && nTiles / p < 4) p--;
    return p;
}

int knn2_parts(int nA, int nB, int dim, int nCU) {
    // train-range parts: spread the query blocks evenly over the CUs (the kernel is VALU-bound,
    // one CU's time is its share of blocks); each part keeps >= 2048 rows
    (void)dim;
    const int nBlk = (nA + 255) / 256;
    int best = 1;
    double bestT = 1e30;
    for (int s = 1; s <= 8; s++) {
        if (s > 1 && nB / s < 2048) break;
        const double t = (double)((nBlk * s + nCU - 1) / nCU) / s;
        if (t < bestT - 1e-9) {
            bestT = t;
            best = s;
        }
    }
    return best;
}

size_t knn2_f32_pairs_bytes(int nB, int dim) {
    size_t nPairs = ((size_t)(nB + 1) / 2 + 1) & ~(size_t)1;
    if (nPairs < 2) nPairs = 2;  // nB = 0: still a (zero) launch grid
    return nPairs * dim * 2 * sizeof(float);
}

void launch_knn2_f32(const float* A, int nA, const float* B, int nB, int dim, int parts, int* partIdx,
                     float* partKey, float* pairs, int* idx, float* key, hipStream_t s) {
    if (nA <= 0) return;
    const int grid = (nA + 255) / 256;
    if (dim != 128 && dim != 64) {
        knn2_f32_generic_kernel<<<grid, 256, 0, s>>>(A, nA, B, nB, dim, idx, key);
        return;
    }
    const int rowsPerPart = parts > 1 ? ((nB + parts - 1) / parts + 1) & ~1 : (nB > 0 ? nB : 1);
    const dim3 g(grid, parts);
    int* oi = parts > 1 ? partIdx : idx;
    float* ok = parts > 1 ? partKey : key;
    const int nPairs = (int)(knn2_f32_pairs_bytes(nB, dim) / (dim * 2 * sizeof(float)));
    const size_t n = (size_t)nPairs * dim * 2;
    f32_row_pairs_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(B, nB, dim, nPairs, pairs);
    if (dim == 128)
        knn2_f32_sgpr_kernel<128><<<g, 256, 0, s>>>(A, nA, pairs, nB, rowsPerPart, oi, ok);
    else
        knn2_f32_sgpr_kernel<64><<<g, 256, 0, s>>>(A, nA, pairs, nB, rowsPerPart, oi, ok);
    if (parts > 1) knn2_f32_merge<<<grid, 256, 0, s>>>(partIdx, partKey, nA, parts, idx, key);
}

void launch_knn2_bits(const uint8_t* A, int nA, const uint8_t* B, int nB, int dimBytes, int parts, int* partIdx,
                      int* partKey, int* idx, int* key, hipStream_t s) {
    if (nA <= 0) return;
    const int grid = (nA + 255) / 256;
    const uint32_t* a = (const uint32_t*)A;
    const uint32_t* b = (const uint32_t*)B;
    const int rowsPerPart = parts > 1 ? (nB + parts - 1) / parts : (nB > 0 ? nB : 1);
    const dim3 g(grid, parts);
    int* oi = parts > 1 ? partIdx : idx;
    int* ok = parts > 1 ? partKey : key;
    switch (dimBytes / 4) {
        case 8: knn2_bits_sgpr_kernel<8><<<g, 256, 0, s>>>(a, nA, b, nB, rowsPerPart, oi, ok); break;
        case 4: knn2_bits_sgpr_kernel<4><<<g, 256, 0, s>>>(a, nA, b, nB, rowsPerPart, oi, ok); break;
        default: knn2_bits_sgpr_kernel<16><<<g, 256, 0, s>>>(a, nA, b, nB, rowsPerPart, oi, ok); break;  // 64 B
    }
    if (parts > 1) knn2_int_merge<<<grid, 256, 0, s>>>(partIdx, partKey, nA, parts, idx, key);
}

int nndr_compact_blocks(int nA) { return nA > 0 ? (nA + 255) / 256 : 1; }

void launch_nndr_compact(int type, const int* idx, const int* key, const float* fkey, const int* partIdx,
                         const int* partKey, int parts, int nA, double eps, int queryOffset, fm3d_dmatch* out,
                         int* count, const LookBack& lb, hipStream_t s) {
    nndr_compact_kernel<<<nndr_compact_blocks(nA), 256, 0, s>>>(type, idx, key, fkey, partIdx, partKey, parts, nA, eps,
                                                              queryOffset, out, count, lb);
}

void launch_nndr(int type, const int* idx, const int* key, const float* fkey, int nA, int nB, double eps,
                 int queryOffset, fm3d_dmatch* knnOut, fm3d_dmatch* cand, int* flag, hipStream_t s) {
    (void)nB;
    if (nA <= 0) return;
    nndr_kernel<<<(nA + 255) / 256, 256, 0, s>>>(type, idx, key, fkey, nA, eps, queryOffset, knnOut, cand, flag);
}

}  // namespace fm3d
