// fm3d_mgpu.cpp -- the hot path over several GPUs of one node, in ONE process, behind the C ABI
// (SURVEY.md §8(b) "fm3d_mgpu_create(ndev, ...) with the same calls", §8(e)).
//
// The reference runs its three stages in one process on one thread (main.cpp:91-155) and has no
// distributed component.  Every stage is independent per query keypoint once frame B's
// descriptors and both image pyramids are on a device, so one frame pair splits into blocks of
// BLOCK queries dealt round-robin over `shares` logical shares, share s belonging to device
// s % ndev.  Per device:
//   * ONE replica: the device's queries (the union of its shares' blocks, in increasing order:
//     local queryIdx) gathered into one array, frame B, its keypoints and both images staged once
//     (pinned H2D) into one context, and ONE pass of the whole path -- one LM launch over all the
//     device's points, so the device pays one end-of-launch tail, not one per share;
//   * exchange: ncclAllGather over xGMI (RCCL, one communicator per device from ncclCommInitAll)
//     of the device's survivor count and its fixed-capacity 64-byte record slot, queued on the
//     device's pipeline stream right after the records (north_star: "RCCL all-gather of per-shard
//     3D points/normals");
//   * merge (plain C++ on the host): device 0's gathered copy, local query indices mapped back
//     through each device's query list, records ordered by query -- byte-identical to one
//     fm3d_pipeline_run of the whole frame pair.
// Four context sets take frame pairs in turn (fm3d_mgpu_submit / fm3d_mgpu_wait), linked in two
// couples (fm3d_pipeline_link: sets 0 -> 1 and 2 -> 3): each device's LM launch takes two frame
// pairs' points, and one couple's staging, front halves and LM workgroups fill the CUs the other's
// launch frees in its tail, as on one GPU (bench.py --gpus N).  Every submit is host-asynchronous:
// one host thread per device gathers its queries and queues its pipeline, then the collectives are
// queued behind the records.
// RCCL is loaded with dlopen on first use, so libfm3d.so itself does not depend on it (a process
// that also loads PyTorch's bundled RCCL keeps one copy per user).
// Test mode FM3D_DEBUG_MGPU_ALIAS=1: a device may be listed more than once (eight "devices" on one
// GPU), so the N-device plan, per-device submit threads, memory pre-flight and merge run on a
// one-GPU box.  RCCL refuses a device twice, so in that mode the all-gather is restated as the same
// copies on the device streams (each destination stream waits for every source's records).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "fm3d.h"
#include "fm3d_internal.h"

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

// ncclGroupStart ... ncclGroupEnd: the group is closed on every path out of the scope, so a failed
// collective never leaves later ones batched into a broken group on this thread
struct RcclGroup {
    bool open = false;
    ncclResult_t start() {
        ncclResult_t r = rccl().groupStart();
        open = r == ncclSuccess;
        return r;
    }
    ncclResult_t end() {
        open = false;
        return rccl().groupEnd();
    }
    ~RcclGroup() {
        if (open) rccl().groupEnd();
    }
};

// the failure text of this thread's last fm3d_mgpu_create (fm3d_mgpu_last_error(NULL))
std::string& create_error() {
    static thread_local std::string e;
    return e;
}

constexpr int kDefaultBlock = 4096;
constexpr int kSets = 4;  // frame pairs in flight (context sets; set 2i joins set 2i + 1's LM launches)

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
    fm3d_ctx* ctx[kSets][16] = {};                 // one context per set and device
    std::vector<ncclComm_t> comms;                  // one per device
    void* send[kSets][16] = {};                     // per set and device: the records (capDev)
    void* recv[kSets][16] = {};                     // ndev x capDev gathered records
    int32_t* cntRecv[kSets][16] = {};               // ndev gathered counts
    int64_t nA = 0, capDev = 0;                     // queries; record capacity per device
    std::vector<std::vector<int32_t>> idx;          // per device: its global query indices (increasing)
    std::vector<std::vector<uint8_t>> rowsA;        // per device: its gathered query rows (host)
    std::vector<std::vector<fm3d_point2f>> kpA;     // per device: its gathered keypoints
    std::vector<fm3d_record> mergeTmp;              // the devices' records before the merge
    std::vector<size_t> memChecked;                 // per device: the memory need last pre-flighted
    bool alias = false;                             // a device listed twice (FM3D_DEBUG_MGPU_ALIAS)
    hipEvent_t aliasEv[kSets][16] = {};             // alias mode: each device's records queued
    bool staged = false;                            // fm3d_mgpu_pipeline_upload ran (set 0)
    bool pending[kSets] = {};
    bool gathered[kSets] = {};                      // the set's all-gather is queued
    int next = 0;                                   // the set the next submit takes
    int waitNext = 0;                               // the set the next wait takes
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

void free_buffers(fm3d_mgpu* m) {
    for (int k = 0; k < kSets; k++)
        for (int d = 0; d < m->ndev; d++) {
            hipSetDevice(m->devices[d]);
            if (m->send[k][d]) hipFree(m->send[k][d]);
            if (m->recv[k][d]) hipFree(m->recv[k][d]);
            if (m->cntRecv[k][d]) hipFree(m->cntRecv[k][d]);
            m->send[k][d] = m->recv[k][d] = nullptr;
            m->cntRecv[k][d] = nullptr;
        }
    m->capDev = 0;
}

size_t row_bytes(int dim, int type) { return type == FM3D_DESC_F32 ? (size_t)dim * 4 : (size_t)dim; }

// the device of block b: share b % shares lives on device share % ndev
int device_of_block(const fm3d_mgpu* m, int64_t b) { return (int)((b % m->shares) % m->ndev); }

// the k-way merge of per-list records (global query indices, each list increasing) under the
// block-cyclic partition: block b's queries all belong to list owner(b), so the merged order is, for
// b = 0, 1, ..., that list's next records below (b + 1) * block.  Returns the records written; a
// record outside its list's blocks is left behind (the caller compares the count).
template <class Owner>
int64_t merge_blocks(const fm3d_record* recs, const int64_t* off, int lists, int64_t nA, int block, Owner owner,
                     fm3d_record* out) {
    std::vector<int64_t> pos(off, off + lists);
    int64_t o = 0;
    const int64_t nb = (nA + block - 1) / block;
    for (int64_t b = 0; b < nb; b++) {
        const int l = owner(b);
        const int64_t lim = std::min<int64_t>((b + 1) * block, nA);
        while (pos[l] < off[l + 1] && recs[pos[l]].queryIdx < lim) out[o++] = recs[pos[l]++];
    }
    return o;
}

// Pre-flight of device memory: before the contexts grow their buffers, every
// device must have room for its four context sets -- each set's LM slabs (the largest launch: any set
// may launch alone) and per-pair buffers (fm3d_internal_memory_need) -- and for the exchange
// buffers, so too little memory is a clean FM3D_ERR_NOMEM, never an allocation failure mid-run.
// `need` grows monotonically; only the growth since the last check must fit in the free memory.
int preflight(fm3d_mgpu* m, int64_t nB, int dim, int type, int width, int height, int64_t capDev) {
    if (m->memChecked.size() != (size_t)m->ndev) m->memChecked.assign(m->ndev, 0);
    std::vector<size_t> need(m->ndev);
    for (int d = 0; d < m->ndev; d++) {
        const int64_t nAd = m->idx.empty() ? 0 : (int64_t)m->idx[d].size();
        size_t per = 0;
        int r = fm3d_internal_memory_need(m->ctx[0][d], nAd, nB, dim, type, width, height, &per);
        if (r) return mfail(m, r, std::string("memory estimate: ") + fm3d_last_error(m->ctx[0][d]));
        need[d] = kSets * (per + (size_t)capDev * sizeof(fm3d_record) * (1 + m->ndev));
    }
    // per physical device (several entries in alias mode): the growth of its entries' needs
    for (int d = 0; d < m->ndev; d++) {
        if (std::find(m->devices.begin(), m->devices.end(), m->devices[d]) - m->devices.begin() != d) continue;
        size_t grow = 0;
        for (int e = d; e < m->ndev; e++)
            if (m->devices[e] == m->devices[d] && need[e] > m->memChecked[e]) grow += need[e] - m->memChecked[e];
        if (!grow) continue;
        size_t freeB = 0, totalB = 0;
        MHIP(m, hipSetDevice(m->devices[d]));
        MHIP(m, hipMemGetInfo(&freeB, &totalB));
        // test hook (tests/test_gpu_parity.py): pretend the device has at most this much free
        if (const char* lim = getenv("FM3D_DEBUG_FREE_MB")) freeB = std::min(freeB, (size_t)strtoull(lim, nullptr, 0) << 20);
        if (grow + ((size_t)256 << 20) > freeB)
            return mfail(m, FM3D_ERR_NOMEM, "device " + std::to_string(m->devices[d]) + ": " +
                                                std::to_string(grow >> 20) + " MiB more needed for " +
                                                std::to_string(kSets) + " context sets (LM slabs + frame-pair "
                                                "buffers), " + std::to_string(freeB >> 20) + " MiB free");
    }
    for (int d = 0; d < m->ndev; d++) m->memChecked[d] = std::max(m->memChecked[d], need[d]);
    return FM3D_OK;
}

// per-device query lists for nA queries; (re)allocates the exchange buffers when they grow
// (nB, dim, type, width, height: the frame pair, for the memory pre-flight)
int plan(fm3d_mgpu* m, int64_t nA, int64_t nB, int dim, int type, int width, int height) {
    m->nA = nA;
    m->idx.assign(m->ndev, {});
    const int64_t nb = (nA + m->block - 1) / m->block;
    for (int64_t b = 0; b < nb; b++) {
        auto& v = m->idx[device_of_block(m, b)];
        for (int64_t q = b * m->block; q < std::min<int64_t>((b + 1) * m->block, nA); q++) v.push_back((int32_t)q);
    }
    int64_t cap = 1;
    for (auto& v : m->idx) cap = std::max<int64_t>(cap, (int64_t)v.size());
    int r;
    if ((r = preflight(m, nB, dim, type, width, height, std::max(cap, m->capDev)))) return r;
    if (cap > m->capDev) {
        free_buffers(m);
        const size_t slot = (size_t)cap * sizeof(fm3d_record);
        for (int k = 0; k < kSets; k++)
            for (int d = 0; d < m->ndev; d++) {
                MHIP(m, hipSetDevice(m->devices[d]));
                MHIP(m, hipMalloc(&m->send[k][d], slot));
                MHIP(m, hipMalloc(&m->recv[k][d], slot * m->ndev));
                MHIP(m, hipMalloc((void**)&m->cntRecv[k][d], sizeof(int32_t) * m->ndev));
            }
        m->capDev = cap;
    }
    return FM3D_OK;
}

// device d's queries gathered into host arrays (local queryIdx = position in m->idx[d])
void gather_device(fm3d_mgpu* m, int d, const void* descA, size_t rb, const fm3d_point2f* kpts1) {
    const auto& ix = m->idx[d];
    m->rowsA[d].resize(ix.size() * rb + 1);
    m->kpA[d].resize(ix.size() + 1);
    for (size_t i = 0; i < ix.size(); i++) {
        std::memcpy(m->rowsA[d].data() + i * rb, (const uint8_t*)descA + (size_t)ix[i] * rb, rb);
        m->kpA[d][i] = kpts1[ix[i]];
    }
}

// the collectives of set k, queued on every device's pipeline stream behind its records
int queue_allgather(fm3d_mgpu* m, int k) {
    const size_t slot = (size_t)m->capDev * sizeof(fm3d_record);
    if (m->alias) {  // test mode: the all-gather's result by copies on the one GPU's streams
        for (int e = 0; e < m->ndev; e++) {
            MHIP(m, hipSetDevice(m->devices[e]));
            MHIP(m, hipEventRecord(m->aliasEv[k][e], fm3d_internal_stream(m->ctx[k][e])));
        }
        for (int d = 0; d < m->ndev; d++) {
            hipStream_t st = fm3d_internal_stream(m->ctx[k][d]);
            MHIP(m, hipSetDevice(m->devices[d]));
            for (int e = 0; e < m->ndev; e++) {
                MHIP(m, hipStreamWaitEvent(st, m->aliasEv[k][e], 0));
                MHIP(m, hipMemcpyAsync(m->cntRecv[k][d] + e, fm3d_internal_kept_dev(m->ctx[k][e]), sizeof(int32_t),
                                       hipMemcpyDeviceToDevice, st));
                MHIP(m, hipMemcpyAsync((char*)m->recv[k][d] + (size_t)e * slot, m->send[k][e], slot,
                                       hipMemcpyDeviceToDevice, st));
            }
        }
        return FM3D_OK;
    }
    RcclGroup g;
    ncclResult_t r = g.start();
    if (r != ncclSuccess) return mfail(m, FM3D_ERR_HIP, std::string("ncclGroupStart: ") + rccl().errStr(r));
    for (int d = 0; d < m->ndev; d++) {
        fm3d_ctx* c = m->ctx[k][d];
        hipStream_t st = fm3d_internal_stream(c);
        r = rccl().allGather(fm3d_internal_kept_dev(c), m->cntRecv[k][d], 1, ncclInt32, m->comms[d], st);
        if (r == ncclSuccess) r = rccl().allGather(m->send[k][d], m->recv[k][d], slot, ncclUint8, m->comms[d], st);
        if (r != ncclSuccess)
            return mfail(m, FM3D_ERR_HIP, "ncclAllGather on device " + std::to_string(m->devices[d]) + ": " +
                                              rccl().errStr(r));
    }
    r = g.end();
    if (r != ncclSuccess) return mfail(m, FM3D_ERR_HIP, std::string("ncclGroupEnd: ") + rccl().errStr(r));
    return FM3D_OK;
}

// wait for set k, then device 0's gathered records -> out in query order
int finish_set(fm3d_mgpu* m, int k, fm3d_record* out, int cap, int* nKept, fm3d_pipeline_stats* stats) {
    std::vector<fm3d_pipeline_stats> st(m->ndev);
    std::vector<int> kept(m->ndev, 0);
    int rc = FM3D_OK;
    for (int d = 0; d < m->ndev; d++) {  // every device's finish runs, so none stays pending
        int r = fm3d_internal_finish(m->ctx[k][d], &kept[d], &st[d]);
        if (r && !rc) rc = mfail(m, r, "device " + std::to_string(m->devices[d]) + ": " + fm3d_last_error(m->ctx[k][d]));
    }
    m->pending[k] = false;
    if (rc) return rc;
    MHIP(m, hipSetDevice(m->devices[0]));
    std::vector<int32_t> cnt(m->ndev);
    MHIP(m, hipMemcpy(cnt.data(), m->cntRecv[k][0], sizeof(int32_t) * m->ndev, hipMemcpyDeviceToHost));
    int64_t total = 0;
    for (int d = 0; d < m->ndev; d++) {
        if (cnt[d] != kept[d]) return mfail(m, FM3D_ERR_HIP, "all-gathered survivor count differs from the device's");
        total += cnt[d];
    }
    if (total > cap) return mfail(m, FM3D_ERR_INVALID, "record buffer too small");
    // every device's list to the host (device 0's gathered copy), local -> global query indices
    std::vector<int64_t> off(m->ndev + 1, 0);
    for (int d = 0; d < m->ndev; d++) off[d + 1] = off[d] + cnt[d];
    m->mergeTmp.resize((size_t)total + 1);
    for (int d = 0; d < m->ndev; d++) {
        if (!cnt[d]) continue;
        fm3d_record* dst = m->mergeTmp.data() + off[d];
        const char* src = (const char*)m->recv[k][0] + (size_t)d * m->capDev * sizeof(fm3d_record);
        MHIP(m, hipMemcpy(dst, src, (size_t)cnt[d] * sizeof(fm3d_record), hipMemcpyDeviceToHost));
        const auto& ix = m->idx[d];
        int32_t prev = -1;
        for (int i = 0; i < cnt[d]; i++) {
            const int32_t l = dst[i].queryIdx;
            if (l < 0 || l >= (int32_t)ix.size() || l <= prev)
                return mfail(m, FM3D_ERR_HIP, "a gathered record carries a bad local query index");
            prev = l;
            dst[i].queryIdx = ix[l];
        }
    }
    // merge in query order without a sort: each device's list is increasing and holds exactly the
    // queries of its blocks, so walking the blocks in order takes, for block b, its device's next
    // records below the block's end (linear in records + blocks)
    const int64_t o = merge_blocks(m->mergeTmp.data(), off.data(), m->ndev, m->nA, m->block,
                                   [m](int64_t b) { return device_of_block(m, b); }, out);
    if (o != total) return mfail(m, FM3D_ERR_HIP, "a gathered record lies outside its device's query blocks");
    if (nKept) *nKept = (int)o;
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        for (int d = 0; d < m->ndev; d++) {
            stats->queries += st[d].queries;
            stats->matches += st[d].matches;
            stats->inliers += st[d].inliers;
            stats->kept += st[d].kept;
            stats->lm.evaluations += st[d].lm.evaluations;
            stats->lm.pixel_evaluations += st[d].lm.pixel_evaluations;
            stats->trains = std::max(stats->trains, st[d].trains);
            // the slowest device (HIP events on its stream: submit -> records)
            stats->total_ms = std::max(stats->total_ms, st[d].total_ms);
            stats->lm_ms = std::max(stats->lm_ms, st[d].lm_ms);
            stats->match_ms = std::max(stats->match_ms, st[d].match_ms);
            stats->pyramid_ms = std::max(stats->pyramid_ms, st[d].pyramid_ms);
        }
        stats->lm.kernel_ms = stats->lm_ms;
    }
    return FM3D_OK;
}

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
    // the shares' records with global query indices, then merged in query order (merge_blocks:
    // block b belongs to share b % shares; every share's list is increasing)
    std::vector<fm3d_record> tmp((size_t)total + 1);
    std::vector<int64_t> off(shares + 1, 0);
    for (int s = 0; s < shares; s++) {
        const int64_t mine = share_count(nA, shares, s, block);
        int32_t prev = -1;
        off[s + 1] = off[s] + counts[s];
        for (int i = 0; i < counts[s]; i++) {
            fm3d_record r = recs[s][i];
            // local index within share s -> (block of the share, offset) -> global query
            if (r.queryIdx < 0 || r.queryIdx >= mine || r.queryIdx <= prev) return FM3D_ERR_INVALID;
            prev = r.queryIdx;
            const int64_t b = r.queryIdx / block, o = r.queryIdx % block;
            r.queryIdx = (int32_t)((b * shares + s) * block + o);
            tmp[off[s] + i] = r;
        }
    }
    const int64_t k = merge_blocks(tmp.data(), off.data(), shares, nA, block,
                                   [shares](int64_t b) { return (int)(b % shares); }, out);
    if (k != total) return FM3D_ERR_INVALID;
    *nOut = (int)k;
    return FM3D_OK;
}

int fm3d_device_count(int* n) {
    if (!n) return FM3D_ERR_INVALID;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    *n = count;
    return FM3D_OK;
}

int fm3d_mgpu_create(const fm3d_settings* s, int ndev, const int* devices, int shares, int block, fm3d_mgpu** out) {
    create_error().clear();
    if (!s || !out || ndev <= 0 || ndev > 16 || shares < ndev || block < 0) return FM3D_ERR_INVALID;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    const char* aliasEnv = getenv("FM3D_DEBUG_MGPU_ALIAS");
    const bool allowAlias = aliasEnv && aliasEnv[0] == '1';
    fm3d_mgpu* m = new fm3d_mgpu();
    m->s = *s;
    m->ndev = ndev;
    m->shares = shares;
    m->block = block ? block : kDefaultBlock;
    for (int d = 0; d < ndev; d++) {
        const int dev = devices ? devices[d] : d;
        const bool twice = std::count(m->devices.begin(), m->devices.end(), dev) != 0;
        if (dev < 0 || dev >= count || (twice && !allowAlias)) {
            delete m;
            return FM3D_ERR_INVALID;  // fewer devices visible than asked for, or a device twice
        }
        m->alias |= twice;
        m->devices.push_back(dev);
    }
    if (!m->alias && !rccl().load()) {
        m->err = rccl().err;
        fm3d_mgpu_destroy(m);
        return FM3D_ERR_UNSUPPORTED;
    }
    for (int k = 0; k < kSets; k++)
        for (int d = 0; d < ndev; d++) {
            int r = fm3d_ctx_create(s, m->devices[d], &m->ctx[k][d]);
            if (!r) r = fm3d_internal_prepare(m->ctx[k][d]);
            if (!r && (k & 1)) r = fm3d_pipeline_link(m->ctx[k - 1][d], m->ctx[k][d]);
            if (r) {
                fm3d_mgpu_destroy(m);
                return r;
            }
        }
    {   // the LM slabs of every context set must fit before anything else is set up
        int r = preflight(m, 0, 128, FM3D_DESC_U8, 0, 0, 0);
        if (r) {
            create_error() = m->err;
            fm3d_mgpu_destroy(m);
            return r;
        }
    }
    if (m->alias) {
        for (int k = 0; k < kSets; k++)
            for (int d = 0; d < ndev; d++)
                if (hipSetDevice(m->devices[d]) != hipSuccess ||
                    hipEventCreateWithFlags(&m->aliasEv[k][d], hipEventDisableTiming) != hipSuccess) {
                    create_error() = "hipEventCreate failed";
                    fm3d_mgpu_destroy(m);
                    return FM3D_ERR_HIP;
                }
    } else {
        m->comms.assign(ndev, nullptr);
        if (rccl().commInitAll(m->comms.data(), ndev, m->devices.data()) != ncclSuccess) {
            fm3d_mgpu_destroy(m);
            return FM3D_ERR_HIP;
        }
    }
    m->rowsA.resize(ndev);
    m->kpA.resize(ndev);
    *out = m;
    return FM3D_OK;
}

void fm3d_mgpu_destroy(fm3d_mgpu* m) {
    if (!m) return;
    for (int k = 0; k < kSets; k++)
        for (int d = 0; d < m->ndev; d++)
            if (m->ctx[k][d]) hipStreamSynchronize(fm3d_internal_stream(m->ctx[k][d]));
    free_buffers(m);
    for (auto c : m->comms)
        if (c) rccl().commDestroy(c);
    for (int k = 0; k < kSets; k++)
        for (int d = 0; d < m->ndev; d++)
            if (m->aliasEv[k][d]) hipEventDestroy(m->aliasEv[k][d]);
    for (int k = 0; k < kSets; k++)
        for (int d = 0; d < m->ndev; d++) fm3d_ctx_destroy(m->ctx[k][d]);
    delete m;
}

const char* fm3d_mgpu_last_error(const fm3d_mgpu* m) { return m ? m->err.c_str() : create_error().c_str(); }

int fm3d_mgpu_set_g12(fm3d_mgpu* m, const double g12[16]) {
    if (!m || !g12) return FM3D_ERR_INVALID;
    for (int k = 0; k < kSets; k++)
        for (int d = 0; d < m->ndev; d++) {
            int r = fm3d_set_g12(m->ctx[k][d], g12);
            if (r) return mfail(m, r, fm3d_last_error(m->ctx[k][d]));
        }
    return FM3D_OK;
}

int fm3d_mgpu_pipeline_upload(fm3d_mgpu* m, const void* descA, int nA, const void* descB, int nB, int dim, int type,
                              const fm3d_point2f* kpts1, const fm3d_point2f* kpts2, const uint8_t* img1,
                              const uint8_t* img2, int width, int height) {
    if (!m || nA < 0 || nB < 0 || dim <= 0 || (nA && (!descA || !kpts1)) || !kpts2) return mfail(m, FM3D_ERR_INVALID, "bad argument");
    for (int k = 0; k < kSets; k++)
        if (m->pending[k]) return mfail(m, FM3D_ERR_INVALID, "a submitted frame pair is pending");
    const size_t rb = row_bytes(dim, type);
    m->staged = false;
    int r;
    if ((r = plan(m, nA, nB, dim, type, width, height))) return r;
    for (int d = 0; d < m->ndev; d++) {
        gather_device(m, d, descA, rb, kpts1);
        const int n = (int)m->idx[d].size();
        r = fm3d_pipeline_upload(m->ctx[0][d], m->rowsA[d].data(), n, descB, nB, dim, type, m->kpA[d].data(), kpts2,
                                 img1, img2, width, height, 0);
        if (r) return mfail(m, r, fm3d_last_error(m->ctx[0][d]));
    }
    m->staged = true;
    return FM3D_OK;
}

int fm3d_mgpu_pipeline_run(fm3d_mgpu* m, fm3d_record* out, int* nKept, fm3d_pipeline_stats* stats) {
    if (!m || !m->staged) return mfail(m, FM3D_ERR_INVALID, "fm3d_mgpu_pipeline_upload not called");
    for (int k = 0; k < kSets; k++)
        if (m->pending[k]) return mfail(m, FM3D_ERR_INVALID, "a submitted frame pair is pending");
    for (int d = 0; d < m->ndev; d++) {
        int r = fm3d_internal_enqueue(m->ctx[0][d], (fm3d_record*)m->send[0][d]);
        if (r) {
            for (int e = 0; e < d; e++) fm3d_internal_finish(m->ctx[0][e], nullptr, nullptr);
            return mfail(m, r, fm3d_last_error(m->ctx[0][d]));
        }
    }
    m->pending[0] = true;
    int r = queue_allgather(m, 0);
    int r2 = finish_set(m, 0, out, (int)m->nA, nKept, stats);
    return r ? r : r2;
}

int fm3d_mgpu_submit(fm3d_mgpu* m, const void* descA, int nA, const void* descB, int nB, int dim, int type,
                     const fm3d_point2f* kpts1, const fm3d_point2f* kpts2, const uint8_t* img1, const uint8_t* img2,
                     int width, int height) {
    if (!m || nA < 0 || nB < 0 || dim <= 0 || (nA && (!descA || !kpts1)) || !kpts2) return mfail(m, FM3D_ERR_INVALID, "bad argument");
    const int k = m->next;
    if (m->pending[k]) return mfail(m, FM3D_ERR_INVALID, "every context set holds a frame pair: fm3d_mgpu_wait first");
    bool others = false;
    for (int j = 0; j < kSets; j++) others |= m->pending[j];
    if (others && nA != m->nA) return mfail(m, FM3D_ERR_INVALID, "frame pairs in flight must have the same query count");
    const size_t rb = row_bytes(dim, type);
    int r;
    // a submit restages set 0 and may re-plan idx / nA: fm3d_mgpu_pipeline_run needs a new upload
    // 
    m->staged = false;
    if (!others && (r = plan(m, nA, nB, dim, type, width, height))) return r;
    if (others && (r = preflight(m, nB, dim, type, width, height, m->capDev))) return r;
    // one host thread per device: gather its queries, stage and queue its path (a member set: its
    // front half; a leader set: the front half, one LM launch with the member set's queued pair,
    // both pairs' records)
    std::vector<int> rc(m->ndev, 0);
    std::vector<std::thread> th;
    for (int d = 0; d < m->ndev; d++)
        th.emplace_back([&, d]() {
            gather_device(m, d, descA, rb, kpts1);
            rc[d] = fm3d_internal_submit_to(m->ctx[k][d], m->rowsA[d].data(), (int)m->idx[d].size(), descB, nB, dim,
                                            type, m->kpA[d].data(), kpts2, img1, img2, width, height,
                                            (fm3d_record*)m->send[k][d]);
        });
    for (auto& t : th) t.join();
    int bad = -1;
    for (int d = 0; d < m->ndev; d++)
        if (rc[d] && bad < 0) bad = d;
    if (bad >= 0) {
        for (int d = 0; d < m->ndev; d++)
            if (!rc[d]) {
                fm3d_internal_flush(m->ctx[k][d]);
                fm3d_internal_finish(m->ctx[k][d], nullptr, nullptr);
            }
        return mfail(m, rc[bad], "device " + std::to_string(m->devices[bad]) + ": " + fm3d_last_error(m->ctx[k][bad]));
    }
    m->pending[k] = true;
    m->gathered[k] = false;
    m->next = (k + 1) % kSets;
    // the all-gathers behind the records now queued: the member set's (its records were queued with
    // this leader's launch) and this set's
    for (int j : {k - 1, k}) {
        if (j < 0 || !m->pending[j] || m->gathered[j] || fm3d_internal_front_only(m->ctx[j][0])) continue;
        if ((r = queue_allgather(m, j))) return r;
        m->gathered[j] = true;
    }
    return FM3D_OK;
}

int fm3d_mgpu_wait(fm3d_mgpu* m, fm3d_record* out, int cap, int* nKept, fm3d_pipeline_stats* stats) {
    if (!m) return FM3D_ERR_INVALID;
    const int k = m->waitNext;
    if (!m->pending[k]) return mfail(m, FM3D_ERR_INVALID, "no frame pair submitted (fm3d_mgpu_submit)");
    m->waitNext = (k + 1) % kSets;
    if (!m->gathered[k]) {  // a member set whose leader set took no pair since: its LM alone
        for (int d = 0; d < m->ndev; d++) {
            int r = fm3d_internal_flush(m->ctx[k][d]);
            if (r) return mfail(m, r, fm3d_last_error(m->ctx[k][d]));
        }
        int r = queue_allgather(m, k);
        if (r) return r;
        m->gathered[k] = true;
    }
    return finish_set(m, k, out, cap, nKept, stats);
}

}  // extern "C"
