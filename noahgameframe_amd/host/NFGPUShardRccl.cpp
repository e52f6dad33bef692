// NFGPUShardRccl.cpp — RCCL transport of the scene shards (include/NFGPUSceneShard.hpp): one rank per
// GPU, rows device to device over xGMI on the world's stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

#include "NFGPUSceneShard.hpp"
#include "nfgpu.h"
#include "nfgpu_shard.h"

namespace nfgpu {

RowMemory DeviceRowMemory() {
    return RowMemory{[](size_t n) {
                         void* p = nullptr;
                         if (hipMalloc(&p, n ? n : 8) != hipSuccess) throw std::runtime_error("hipMalloc (shard rows)");
                         return p;
                     },
                     [](void* p) { (void)hipFree(p); },
                     // complete when it returns: a device-to-device hipMemcpy may return before the
                     // copy is done, and the rows' readers (the import's copy on the world's stream,
                     // the source's next export) are not ordered after the null stream
                     [](void* d, const void* s, size_t n) {
                         if (hipMemcpyAsync(d, s, n, hipMemcpyDeviceToDevice, nullptr) != hipSuccess ||
                             hipStreamSynchronize(nullptr) != hipSuccess)
                             throw std::runtime_error("hipMemcpy (shard rows)");
                     }};
}

static void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

std::vector<uint8_t> RcclTransport::NewUniqueId() {
    ncclUniqueId id;
    nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return std::vector<uint8_t>((const uint8_t*)&id, (const uint8_t*)&id + sizeof id);
}

RcclTransport::RcclTransport(const std::vector<uint8_t>& unique_id, int rank, int size, void* stream)
    : stream_(stream), rank_(rank), size_(size) {
    if (unique_id.size() != sizeof(ncclUniqueId)) throw std::runtime_error("RcclTransport: bad unique id");
    if (hipGetDevice(&device_) != hipSuccess) throw std::runtime_error("RcclTransport: hipGetDevice");
    ncclUniqueId id;
    memcpy(&id, unique_id.data(), sizeof id);
    ncclComm_t c = nullptr, m = nullptr;
    nccl_check(ncclCommInitRank(&c, size, id, rank), "ncclCommInitRank");
    comm_ = c;
    // the tickets' channel: a communicator of the same ranks and a stream of its own
    nccl_check(ncclCommSplit(c, 0, rank, &m, nullptr), "ncclCommSplit");
    meta_comm_ = m;
    hipStream_t ms = nullptr;
    if (hipStreamCreateWithFlags(&ms, hipStreamNonBlocking) != hipSuccess)
        throw std::runtime_error("RcclTransport: hipStreamCreate");
    meta_stream_ = ms;
}

void RcclTransport::Abort() {
    // (a collective blocked on a peer that never arrives returns; the communicators are gone).  The
    // handles are not reset here: the gather thread may be reading them; it sees aborted_ instead
    if (aborted_.exchange(true)) return;
    if (meta_comm_) (void)ncclCommAbort((ncclComm_t)meta_comm_);
    if (comm_) (void)ncclCommAbort((ncclComm_t)comm_);
}

RcclTransport::~RcclTransport() {
    if (buf_) (void)hipFree(buf_);
    if (!aborted_.load()) {  // (aborted communicators were released by ncclCommAbort)
        if (meta_comm_) (void)ncclCommDestroy((ncclComm_t)meta_comm_);
        if (comm_) (void)ncclCommDestroy((ncclComm_t)comm_);
    }
    if (meta_stream_) (void)hipStreamDestroy((hipStream_t)meta_stream_);
}

// tickets: every rank's count, then every rank's rows padded to the largest count (two all-gathers
// of device buffers on the tickets' communicator and stream; tickets are small).  May run on a
// worker thread (SceneShard::EndFrame): the HIP device is per thread.
int RcclTransport::AllGather(const std::vector<int64_t>& mine, std::vector<int64_t>& all) {
    if (aborted_.load() || hipSetDevice(device_) != hipSuccess) return NFK_ERR_HIP;
    hipStream_t s = (hipStream_t)meta_stream_;
    auto reserve = [&](size_t words) {
        if (words <= buf_cap_) return true;
        if (buf_) (void)hipFree(buf_);
        buf_cap_ = words + words / 2 + 64;
        return hipMalloc((void**)&buf_, buf_cap_ * 8) == hipSuccess;
    };
    if (!reserve((size_t)2 * size_)) return NFK_ERR_HIP;
    const int64_t n = (int64_t)mine.size();
    if (hipMemcpyAsync(buf_, &n, 8, hipMemcpyHostToDevice, s) != hipSuccess) return NFK_ERR_HIP;
    if (ncclAllGather(buf_, buf_ + size_, 1, ncclInt64, (ncclComm_t)meta_comm_, s) != ncclSuccess) return NFK_ERR_HIP;
    std::vector<int64_t> counts(size_);
    if (hipMemcpyAsync(counts.data(), buf_ + size_, 8 * (size_t)size_, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return NFK_ERR_HIP;
    int64_t mx = 0;
    for (int64_t c : counts) mx = std::max(mx, c);
    all.clear();
    if (mx == 0) return NFK_OK;
    if (aborted_.load() || !reserve((size_t)mx * (1 + size_))) return NFK_ERR_HIP;
    if ((n && hipMemcpyAsync(buf_, mine.data(), (size_t)n * 8, hipMemcpyHostToDevice, s) != hipSuccess) ||
        ncclAllGather(buf_, buf_ + mx, (size_t)mx, ncclInt64, (ncclComm_t)meta_comm_, s) != ncclSuccess)
        return NFK_ERR_HIP;
    std::vector<int64_t> padded((size_t)mx * size_);
    if (hipMemcpyAsync(padded.data(), buf_ + mx, padded.size() * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return NFK_ERR_HIP;
    for (int r = 0; r < size_; r++) all.insert(all.end(), padded.begin() + (size_t)r * mx, padded.begin() + (size_t)r * mx + counts[r]);
    return NFK_OK;
}

// rows: grouped ncclSend / ncclRecv on the stream the rows were packed on (the world's, which
// SceneShard passes), so the unpack that follows on it is ordered after the receive
int RcclTransport::AllToAllV(const uint64_t* send, const std::vector<size_t>& scount, uint64_t* recv,
                             const std::vector<size_t>& rcount, void* stream) {
    if (aborted_.load()) return NFK_ERR_HIP;
    hipStream_t s = (hipStream_t)(stream ? stream : stream_);
    size_t so = 0, ro = 0;
    if (ncclGroupStart() != ncclSuccess) return NFK_ERR_HIP;
    bool ok = true;
    for (int r = 0; r < size_ && ok; r++) {
        if (scount[r] && ncclSend(send + so, scount[r], ncclUint64, r, (ncclComm_t)comm_, s) != ncclSuccess) ok = false;
        if (ok && rcount[r] && ncclRecv(recv + ro, rcount[r], ncclUint64, r, (ncclComm_t)comm_, s) != ncclSuccess)
            ok = false;
        so += scount[r];
        ro += rcount[r];
    }
    // (the group is always closed: an open group would leave the communicator unusable)
    if (ncclGroupEnd() != ncclSuccess) ok = false;
    return ok ? NFK_OK : NFK_ERR_HIP;
}

}  // namespace nfgpu

// ---------------- C-ABI (include/nfgpu_shard.h) ----------------
namespace {
struct CShard {
    std::unique_ptr<nfgpu::RcclTransport> t;
    std::unique_ptr<nfgpu::SceneShard> s;
    std::vector<int32_t> owner;
    std::vector<nfgpu::Ticket> recv;
};
}  // namespace

extern "C" {

int nfs_rccl_unique_id(uint8_t* id128) {
    if (!id128) return NFK_ERR_ARG;
    try {
        const std::vector<uint8_t> id = nfgpu::RcclTransport::NewUniqueId();
        if (id.size() != 128) return NFK_ERR_STATE;
        memcpy(id128, id.data(), 128);
        return NFK_OK;
    } catch (const std::exception&) {
        return NFK_ERR_HIP;
    }
}

int nfs_create_rccl(void* world, const uint8_t* id128, int32_t rank, int32_t size, const int32_t* owner,
                    int32_t n_scenes, int32_t pid_scene, int32_t pid_group, int32_t pid_x, int32_t pid_y,
                    int32_t pid_z, int32_t exchange_every, void** shard) {
    if (!world || !id128 || !owner || n_scenes <= 0 || !shard || rank < 0 || rank >= size) return NFK_ERR_ARG;
    try {
        auto c = std::make_unique<CShard>();
        c->owner.assign(owner, owner + n_scenes);
        void* stream = nullptr;
        if (nfk_get_stream(world, &stream)) return NFK_ERR_ARG;
        c->t = std::make_unique<nfgpu::RcclTransport>(std::vector<uint8_t>(id128, id128 + 128), rank, size, stream);
        const std::vector<int32_t>* own = &c->owner;
        c->s = std::make_unique<nfgpu::SceneShard>(
            world, c->t.get(),
            [own](int scene) { return scene >= 0 && scene < (int)own->size() ? (*own)[(size_t)scene] : -1; },
            pid_scene, pid_group, pid_x, pid_y, pid_z, nfgpu::DeviceRowMemory(), stream);
        c->s->SetExchangeEvery(exchange_every);
        *shard = c.release();
        return NFK_OK;
    } catch (const std::exception&) {
        return NFK_ERR_HIP;
    }
}

void nfs_destroy(void* shard) { delete (CShard*)shard; }

int nfs_queue_switch(void* shard, int32_t n, const int64_t* gh, const int64_t* gd, const int32_t* cls,
                     const int32_t* pl, const int32_t* scene, const int32_t* group, const float* x, const float* y,
                     const float* z) {
    CShard* c = (CShard*)shard;
    if (!c || n < 0) return NFK_ERR_ARG;
    for (int32_t i = 0; i < n; i++) {
        if (c->s->Owner(scene[i]) < 0) return NFK_ERR_ARG;  // a scene no rank owns
        c->s->QueueSwitch(gh[i], gd[i], cls[i], pl[i], scene[i], group[i], x[i], y[i], z[i]);
    }
    return NFK_OK;
}

int nfs_begin_frame(void* shard, int64_t* n_sent, int64_t* n_received) {
    CShard* c = (CShard*)shard;
    if (!c) return NFK_ERR_ARG;
    std::vector<nfgpu::Ticket> sent;
    const int r = c->s->BeginFrame(&sent, &c->recv);
    if (n_sent) *n_sent = (int64_t)sent.size();
    if (n_received) *n_received = (int64_t)c->recv.size();
    return r;
}

int nfs_received(void* shard, int64_t cap, int64_t* gh, int64_t* gd, int32_t* cls, int32_t* pl, int32_t* scene,
                 int32_t* group) {
    CShard* c = (CShard*)shard;
    if (!c) return NFK_ERR_ARG;
    for (size_t i = 0; i < c->recv.size() && (int64_t)i < cap; i++) {
        const nfgpu::Ticket& k = c->recv[i];
        gh[i] = k.guid_head;
        gd[i] = k.guid_data;
        cls[i] = k.cls;
        pl[i] = k.is_player;
        scene[i] = k.scene;
        group[i] = k.group;
    }
    return NFK_OK;
}

int nfs_end_frame(void* shard) {
    CShard* c = (CShard*)shard;
    return c ? c->s->EndFrame() : NFK_ERR_ARG;
}

int nfs_stats(void* shard, int64_t* out4) {
    CShard* c = (CShard*)shard;
    if (!c || !out4) return NFK_ERR_ARG;
    out4[0] = c->s->migrated_out;
    out4[1] = c->s->migrated_in;
    out4[2] = c->s->transport_calls;
    out4[3] = c->s->frames;
    return NFK_OK;
}

int nfs_rank_top(void* shard, int32_t pid, int32_t k, int32_t* n_out, int64_t* gh, int64_t* gd, double* score) {
    CShard* c = (CShard*)shard;
    if (!c || !n_out || k < 0) return NFK_ERR_ARG;
    std::vector<nfgpu::SceneShard::RankRow> rows;
    const int r = c->s->RankTop(pid, k, &rows);
    *n_out = (int32_t)rows.size();
    for (size_t i = 0; i < rows.size(); i++) {
        gh[i] = rows[i].guid_head;
        gd[i] = rows[i].guid_data;
        score[i] = rows[i].score;
    }
    return r;
}
}  // extern "C"
