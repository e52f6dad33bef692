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
    if (host_) (void)hipHostFree(host_);
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
        if (words > buf_cap_) {
            if (buf_) (void)hipFree(buf_);
            buf_ = nullptr;
            buf_cap_ = words + words / 2 + 64;
            if (hipMalloc((void**)&buf_, buf_cap_ * 8) != hipSuccess) return false;
        }
        if (words > host_cap_) {
            if (host_) (void)hipHostFree(host_);
            host_ = nullptr;
            host_cap_ = words + words / 2 + 64;
            if (hipHostMalloc((void**)&host_, host_cap_ * 8, hipHostMallocDefault) != hipSuccess) return false;
        }
        return true;
    };
    // round 1: [count, the first W words] from every rank (W the same on every rank)
    const size_t W = w_first_, R = 1 + W;
    const int64_t n = (int64_t)mine.size();
    const size_t n1 = std::min((size_t)n, W);
    if (!reserve(R * (1 + (size_t)size_))) return NFK_ERR_HIP;
    host_[0] = n;
    if (n1) memcpy(host_ + 1, mine.data(), n1 * 8);
    if (n1 < W) memset(host_ + 1 + n1, 0, (W - n1) * 8);
    if (hipMemcpyAsync(buf_, host_, R * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        ncclAllGather(buf_, buf_ + R, R, ncclInt64, (ncclComm_t)meta_comm_, s) != ncclSuccess ||
        hipMemcpyAsync(host_ + R, buf_ + R, R * (size_t)size_ * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return NFK_ERR_HIP;
    std::vector<int64_t> counts((size_t)size_);
    int64_t mx = 0;
    for (int r = 0; r < size_; r++) {
        counts[(size_t)r] = host_[R + (size_t)r * R];
        mx = std::max(mx, counts[(size_t)r]);
    }
    std::vector<int64_t> first(host_ + R, host_ + R + R * (size_t)size_);  // (host_ is reused below)
    all.clear();
    if ((size_t)mx <= W) {
        for (int r = 0; r < size_; r++)
            all.insert(all.end(), first.begin() + (size_t)r * R + 1, first.begin() + (size_t)r * R + 1 + (size_t)counts[(size_t)r]);
    } else {
        // round 2: the words past W, padded to the largest remainder
        const size_t T = (size_t)mx - W;
        if (aborted_.load() || !reserve(T * (1 + (size_t)size_))) return NFK_ERR_HIP;
        const size_t n2 = (size_t)n > W ? (size_t)n - W : 0;
        if (n2) memcpy(host_, mine.data() + W, n2 * 8);
        if (n2 < T) memset(host_ + n2, 0, (T - n2) * 8);
        if (hipMemcpyAsync(buf_, host_, T * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
            ncclAllGather(buf_, buf_ + T, T, ncclInt64, (ncclComm_t)meta_comm_, s) != ncclSuccess ||
            hipMemcpyAsync(host_ + T, buf_ + T, T * (size_t)size_ * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return NFK_ERR_HIP;
        for (int r = 0; r < size_; r++) {
            const size_t c = (size_t)counts[(size_t)r];
            all.insert(all.end(), first.begin() + (size_t)r * R + 1, first.begin() + (size_t)r * R + 1 + std::min(c, W));
            if (c > W) all.insert(all.end(), host_ + T + (size_t)r * T, host_ + T + (size_t)r * T + (c - W));
        }
    }
    // the next first round holds this gather's largest list (up to 64k words, 512 KB per rank)
    while (w_first_ < (size_t)mx && w_first_ < ((size_t)1 << 16)) w_first_ *= 2;
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
