// fm3d_mgpu.cpp -- the hot path over several GPUs of one node, in ONE process, behind the C ABI
// (SURVEY.md §8(b) "fm3d_mgpu_create(ndev, ...) with the same calls", §8(e)).
//
// The reference runs its three stages in one process on one thread (main.cpp:91-155) and has no
// distributed component.  Every stage is independent per query keypoint once frame B's
// descriptors and both image pyramids are on a device, so one frame pair splits into logical
// shares of query blocks (BLOCK queries each, dealt round-robin over the shares: every share sees
// the same mix of queries), share s running on devices[s % ndev]:
//   * upload: each share's queries gathered into one array (local queryIdx), frame B, keypoints
//     of frame B and both images replicated to its device (host uploads, one context per share);
//   * run: one host thread per device runs that device's shares one after the other (the LM
//     kernel is persistent and fills the GPU), each writing its survivor records straight into
//     its slot of the device's all-gather send buffer;
//   * exchange: ncclAllGather over xGMI (RCCL, one communicator per device from ncclCommInitAll)
//     of the per-share survivor counts and of the fixed-capacity 64-byte record slots, so every
//     device holds every share's records (north_star: "RCCL all-gather of per-shard 3D
//     points/normals");
//   * merge (fm3d_merge_shares, plain C++ on the host): local query indices mapped back to
//     global ones in closed form, records ordered by query -- byte-identical to one
//     fm3d_pipeline_run of the whole frame pair.
// RCCL is loaded with dlopen on first use, so libfm3d.so itself does not depend on it (a process
// that also loads PyTorch's bundled RCCL keeps one copy per user).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "fm3d.h"

namespace {

struct Rccl {
    void* h = nullptr;
    ncclResult_t (*commInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*allGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*groupStart)() = nullptr;
    ncclResult_t (*groupEnd)() = nullptr;
    const char* (*errStr)(ncclResult_t) = nullptr;
    std::string err;
    bool load() {
        if (h) return true;
        const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        for (const char* n : names)
            if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) {
            err = std::string("cannot load RCCL (librccl.so.1): ") + dlerror();
            return false;
        }
        commInitAll = (decltype(commInitAll))dlsym(h, "ncclCommInitAll");
        commDestroy = (decltype(commDestroy))dlsym(h, "ncclCommDestroy");
        allGather = (decltype(allGather))dlsym(h, "ncclAllGather");
        groupStart = (decltype(groupStart))dlsym(h, "ncclGroupStart");
        groupEnd = (decltype(groupEnd))dlsym(h, "ncclGroupEnd");
        errStr = (decltype(errStr))dlsym(h, "ncclGetErrorString");
        if (!commInitAll || !commDestroy || !allGather || !groupStart || !groupEnd || !errStr) {
            err = "RCCL library lacks an entry point";
            dlclose(h);
            h = nullptr;
            return false;
        }
        return true;
    }
};

Rccl& rccl() {
    static Rccl r;
    return r;
}

constexpr int kDefaultBlock = 4096;

// number of queries of share s under the block-cyclic partition
int64_t share_count(int64_t nA, int shares, int s, int block) {
    const int64_t nb = (nA + block - 1) / block;  // blocks
    int64_t cnt = 0;
    for (int64_t b = s; b < nb; b += shares) cnt += std::min<int64_t>(block, nA - b * block);
    return cnt;
}

}  // namespace

struct fm3d_mgpu {
    fm3d_settings s{};
    int ndev = 0, shares = 0, block = kDefaultBlock;
    std::vector<int> devices;
    std::vector<fm3d_ctx*> ctx;           // one per share
    std::vector<ncclComm_t> comms;        // one per device
    std::vector<hipStream_t> streams;     // one per device (the collectives)
    std::vector<void*> send, recv;        // per device: L slots x cap records / ndev x L slots
    std::vector<int32_t*> cntSend, cntRecv;
    int64_t nA = 0, cap = 0;              // queries; records per share slot
    std::vector<int> nq;                  // queries per share
    int L = 0;                            // share slots per device (ceil(shares / ndev))
    bool staged = false;
    std::string err;
};

namespace {

int mfail(fm3d_mgpu* m, int code, const std::string& msg) {
    if (m) m->err = msg;
    return code;
}

#define MHIP(m, x)                                                                              \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) return mfail(m, FM3D_ERR_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

#define MNCCL(m, x)                                                                             \
    do {                                                                                        \
        ncclResult_t r_ = (x);                                                                  \
        if (r_ != ncclSuccess) return mfail(m, FM3D_ERR_HIP, std::string(#x ": ") + rccl().errStr(r_)); \
    } while (0)

void free_buffers(fm3d_mgpu* m) {
    for (int d = 0; d < (int)m->send.size(); d++) {
        hipSetDevice(m->devices[d]);
        if (m->send[d]) hipFree(m->send[d]);
        if (m->recv[d]) hipFree(m->recv[d]);
        if (m->cntSend[d]) hipFree(m->cntSend[d]);
        if (m->cntRecv[d]) hipFree(m->cntRecv[d]);
        m->send[d] = m->recv[d] = nullptr;
        m->cntSend[d] = m->cntRecv[d] = nullptr;
    }
}

size_t row_bytes(int dim, int type) { return type == FM3D_DESC_F32 ? (size_t)dim * 4 : (size_t)dim; }

}  // namespace

extern "C" {

int fm3d_share_queries(int nA, int shares, int s, int block, int32_t* idx, int cap, int* n) {
    if (nA < 0 || shares <= 0 || s < 0 || s >= shares || block <= 0 || !n) return FM3D_ERR_INVALID;
    const int64_t cnt = share_count(nA, shares, s, block);
    *n = (int)cnt;
    if (!idx) return FM3D_OK;
    if (cap < cnt) return FM3D_ERR_INVALID;
    int64_t k = 0;
    for (int64_t b = s; b * block < nA; b += shares)
        for (int64_t q = b * block; q < std::min<int64_t>((b + 1) * block, nA); q++) idx[k++] = (int32_t)q;
    return FM3D_OK;
}

int fm3d_merge_shares(int nA, int shares, int block, const fm3d_record* const* recs, const int* counts,
                      fm3d_record* out, int* nOut) {
    if (nA < 0 || shares <= 0 || block <= 0 || !recs || !counts || !nOut) return FM3D_ERR_INVALID;
    int64_t total = 0;
    for (int s = 0; s < shares; s++) {
        if (counts[s] < 0 || (counts[s] && !recs[s])) return FM3D_ERR_INVALID;
        total += counts[s];
    }
    if (total > nA || (total && !out)) return FM3D_ERR_INVALID;
    int64_t k = 0;
    for (int s = 0; s < shares; s++) {
        const int64_t mine = share_count(nA, shares, s, block);
        int32_t prev = -1;
        for (int i = 0; i < counts[s]; i++) {
            fm3d_record r = recs[s][i];
            // local index within share s -> (block of the share, offset) -> global query
            if (r.queryIdx < 0 || r.queryIdx >= mine || r.queryIdx <= prev) return FM3D_ERR_INVALID;
            prev = r.queryIdx;
            const int64_t b = r.queryIdx / block, o = r.queryIdx % block;
            r.queryIdx = (int32_t)((b * shares + s) * block + o);
            out[k++] = r;
        }
    }
    // every share's list is in increasing query order and the query sets are disjoint: the
    // merged list is the records ordered by queryIdx (one record per query at most)
    std::sort(out, out + k, [](const fm3d_record& a, const fm3d_record& b) { return a.queryIdx < b.queryIdx; });
    *nOut = (int)k;
    return FM3D_OK;
}

int fm3d_mgpu_create(const fm3d_settings* s, int ndev, const int* devices, int shares, int block, fm3d_mgpu** out) {
    if (!s || !out || ndev <= 0 || shares < ndev || block < 0) return FM3D_ERR_INVALID;
    *out = nullptr;
    fm3d_mgpu* m = new fm3d_mgpu();
    m->s = *s;
    m->ndev = ndev;
    m->shares = shares;
    m->block = block ? block : kDefaultBlock;
    m->L = (shares + ndev - 1) / ndev;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    for (int d = 0; d < ndev; d++) {
        const int dev = devices ? devices[d] : d;
        if (dev < 0 || dev >= count) {
            delete m;
            return FM3D_ERR_INVALID;
        }
        m->devices.push_back(dev);
    }
    if (!rccl().load()) {
        m->err = rccl().err;
        fm3d_mgpu_destroy(m);
        return FM3D_ERR_UNSUPPORTED;
    }
    m->ctx.assign(shares, nullptr);
    for (int j = 0; j < shares; j++) {
        int r = fm3d_ctx_create(s, m->devices[j % ndev], &m->ctx[j]);
        if (r) {
            fm3d_mgpu_destroy(m);
            return r;
        }
    }
    m->comms.assign(ndev, nullptr);
    if (rccl().commInitAll(m->comms.data(), ndev, m->devices.data()) != ncclSuccess) {
        fm3d_mgpu_destroy(m);
        return FM3D_ERR_HIP;
    }
    m->streams.assign(ndev, nullptr);
    m->send.assign(ndev, nullptr);
    m->recv.assign(ndev, nullptr);
    m->cntSend.assign(ndev, nullptr);
    m->cntRecv.assign(ndev, nullptr);
    for (int d = 0; d < ndev; d++) {
        hipSetDevice(m->devices[d]);
        if (hipStreamCreateWithFlags(&m->streams[d], hipStreamNonBlocking) != hipSuccess) {
            fm3d_mgpu_destroy(m);
            return FM3D_ERR_HIP;
        }
    }
    *out = m;
    return FM3D_OK;
}

void fm3d_mgpu_destroy(fm3d_mgpu* m) {
    if (!m) return;
    free_buffers(m);
    for (size_t d = 0; d < m->streams.size(); d++)
        if (m->streams[d]) {
            hipSetDevice(m->devices[d]);
            hipStreamDestroy(m->streams[d]);
        }
    for (auto c : m->comms)
        if (c) rccl().commDestroy(c);
    for (auto c : m->ctx) fm3d_ctx_destroy(c);
    delete m;
}

const char* fm3d_mgpu_last_error(const fm3d_mgpu* m) { return m ? m->err.c_str() : "null handle"; }

int fm3d_mgpu_set_g12(fm3d_mgpu* m, const double g12[16]) {
    if (!m || !g12) return FM3D_ERR_INVALID;
    for (auto c : m->ctx) {
        int r = fm3d_set_g12(c, g12);
        if (r) return mfail(m, r, fm3d_last_error(c));
    }
    return FM3D_OK;
}

int fm3d_mgpu_pipeline_upload(fm3d_mgpu* m, const void* descA, int nA, const void* descB, int nB, int dim, int type,
                              const fm3d_point2f* kpts1, const fm3d_point2f* kpts2, const uint8_t* img1,
                              const uint8_t* img2, int width, int height) {
    if (!m || nA < 0 || nB < 0 || dim <= 0 || (nA && (!descA || !kpts1)) || !kpts2) return mfail(m, FM3D_ERR_INVALID, "bad argument");
    const size_t rb = row_bytes(dim, type);
    free_buffers(m);
    m->staged = false;
    m->nA = nA;
    m->cap = 1;
    for (int j = 0; j < m->shares; j++) m->cap = std::max<int64_t>(m->cap, share_count(nA, m->shares, j, m->block));
    m->nq.assign(m->shares, 0);
    std::vector<int32_t> idx;
    std::vector<uint8_t> a;
    std::vector<fm3d_point2f> k1;
    for (int j = 0; j < m->shares; j++) {
        int n = 0;
        fm3d_share_queries(nA, m->shares, j, m->block, nullptr, 0, &n);
        m->nq[j] = n;
        if (n == 0) continue;  // more shares than blocks: nothing to stage or run
        idx.resize(n);
        fm3d_share_queries(nA, m->shares, j, m->block, idx.data(), n, &n);
        a.resize((size_t)n * rb + 1);
        k1.resize((size_t)n + 1);
        for (int i = 0; i < n; i++) {
            std::memcpy(a.data() + (size_t)i * rb, (const uint8_t*)descA + (size_t)idx[i] * rb, rb);
            k1[i] = kpts1[idx[i]];
        }
        int r = fm3d_pipeline_upload(m->ctx[j], a.data(), n, descB, nB, dim, type, k1.data(), kpts2, img1, img2, width,
                                     height, 0);
        if (r) return mfail(m, r, fm3d_last_error(m->ctx[j]));
    }
    const size_t slot = (size_t)m->cap * sizeof(fm3d_record);
    for (int d = 0; d < m->ndev; d++) {
        hipSetDevice(m->devices[d]);
        MHIP(m, hipMalloc(&m->send[d], slot * m->L));
        MHIP(m, hipMalloc(&m->recv[d], slot * m->L * m->ndev));
        MHIP(m, hipMalloc((void**)&m->cntSend[d], sizeof(int32_t) * m->L));
        MHIP(m, hipMalloc((void**)&m->cntRecv[d], sizeof(int32_t) * m->L * m->ndev));
        MHIP(m, hipMemset(m->cntSend[d], 0, sizeof(int32_t) * m->L));
    }
    m->staged = true;
    return FM3D_OK;
}

int fm3d_mgpu_pipeline_run(fm3d_mgpu* m, fm3d_record* out, int* nKept, fm3d_pipeline_stats* stats) {
    if (!m || !m->staged) return mfail(m, FM3D_ERR_INVALID, "fm3d_mgpu_pipeline_upload not called");
    const size_t slot = (size_t)m->cap * sizeof(fm3d_record);
    std::vector<int> kept(m->shares, 0), rc(m->shares, 0);
    std::vector<fm3d_pipeline_stats> st(m->shares);
    std::vector<double> devMs(m->ndev, 0.0);
    // one host thread per device; a device's shares run one after the other
    std::vector<std::thread> th;
    for (int d = 0; d < m->ndev; d++)
        th.emplace_back([m, d, slot, &kept, &rc, &st, &devMs]() {
            for (int j = d, l = 0; j < m->shares; j += m->ndev, l++) {
                fm3d_record* dst = (fm3d_record*)((char*)m->send[d] + (size_t)l * slot);
                if (m->nq[j] == 0) continue;
                rc[j] = fm3d_pipeline_run(m->ctx[j], dst, &kept[j], &st[j]);
                if (rc[j]) return;
                devMs[d] += st[j].total_ms;
            }
        });
    for (auto& t : th) t.join();
    for (int j = 0; j < m->shares; j++)
        if (rc[j]) return mfail(m, rc[j], fm3d_last_error(m->ctx[j]));
    // counts per slot (empty slots of the last device keep 0), then the RCCL all-gathers
    for (int d = 0; d < m->ndev; d++) {
        std::vector<int32_t> c(m->L, 0);
        for (int j = d, l = 0; j < m->shares; j += m->ndev, l++) c[l] = kept[j];
        hipSetDevice(m->devices[d]);
        MHIP(m, hipMemcpyAsync(m->cntSend[d], c.data(), sizeof(int32_t) * m->L, hipMemcpyHostToDevice, m->streams[d]));
        MHIP(m, hipStreamSynchronize(m->streams[d]));
    }
    MNCCL(m, rccl().groupStart());
    for (int d = 0; d < m->ndev; d++) {
        MNCCL(m, rccl().allGather(m->cntSend[d], m->cntRecv[d], (size_t)m->L, ncclInt32, m->comms[d], m->streams[d]));
        MNCCL(m, rccl().allGather(m->send[d], m->recv[d], slot * m->L, ncclUint8, m->comms[d], m->streams[d]));
    }
    MNCCL(m, rccl().groupEnd());
    for (int d = 0; d < m->ndev; d++) {
        hipSetDevice(m->devices[d]);
        MHIP(m, hipStreamSynchronize(m->streams[d]));
    }
    // device 0's copy of every share's records -> host, merged in query order
    hipSetDevice(m->devices[0]);
    std::vector<int32_t> cnt((size_t)m->L * m->ndev);
    MHIP(m, hipMemcpy(cnt.data(), m->cntRecv[0], sizeof(int32_t) * cnt.size(), hipMemcpyDeviceToHost));
    std::vector<std::vector<fm3d_record>> part(m->shares);
    std::vector<const fm3d_record*> ptrs(m->shares);
    std::vector<int> counts(m->shares);
    for (int j = 0; j < m->shares; j++) {
        const int d = j % m->ndev, l = j / m->ndev;
        const int c = cnt[(size_t)d * m->L + l];
        if (c != kept[j]) return mfail(m, FM3D_ERR_HIP, "all-gathered survivor count differs from the share's");
        part[j].resize((size_t)c + 1);
        const char* src = (const char*)m->recv[0] + ((size_t)d * m->L + l) * slot;
        if (c) MHIP(m, hipMemcpy(part[j].data(), src, (size_t)c * sizeof(fm3d_record), hipMemcpyDeviceToHost));
        ptrs[j] = part[j].data();
        counts[j] = c;
    }
    int n = 0;
    int r = fm3d_merge_shares((int)m->nA, m->shares, m->block, ptrs.data(), counts.data(), out, &n);
    if (r) return mfail(m, r, "merge of the gathered shares failed");
    if (nKept) *nKept = n;
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        for (int j = 0; j < m->shares; j++) {
            stats->queries += st[j].queries;
            stats->matches += st[j].matches;
            stats->inliers += st[j].inliers;
            stats->kept += st[j].kept;
            stats->lm.evaluations += st[j].lm.evaluations;
            stats->lm.pixel_evaluations += st[j].lm.pixel_evaluations;
        }
        for (int j = 0; j < m->shares; j++) stats->trains = std::max(stats->trains, st[j].trains);
        stats->total_ms = *std::max_element(devMs.begin(), devMs.end());  // the slowest device
    }
    return FM3D_OK;
}

}  // extern "C"
