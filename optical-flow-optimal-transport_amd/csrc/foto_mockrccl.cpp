// In-process RCCL transport for tests (libfoto_mockrccl.so only; the product library links
// the real librccl).  RCCL refuses two ranks on one GPU ("Duplicate GPU detected") and the test
// pool has one GPU per box, so the RCCL branches of foto_bb.cpp (grouped ncclSend/ncclRecv
// exchanges, the in-place ncclAllGather of the s-step moments, ncclCommInitRank) cannot run on
// real RCCL before the 8-GPU node does.  This file implements exactly the calls libfoto makes,
// with NCCL's semantics, for W ranks that are W host threads of one process sharing device 0:
//   * ncclSend / ncclRecv inside ncclGroupStart / ncclGroupEnd: the k-th send from rank a to
//     rank b is matched with the k-th receive posted by b from a (NCCL's rule).  A matched pair
//     becomes a device copy on the receiver's stream, ordered after the sender's stream reached
//     the send (event) and before the receiver's stream moves on; the sender's stream waits for
//     the copy before it can overwrite the buffer.  ncclGroupEnd returns once every operation
//     of the group is matched (every copy is enqueued), as RCCL's enqueue completes.
//   * ncclAllGather (in place): the k-th call of every rank forms one collective; each rank's
//     stream receives every other rank's slot, and every rank's stream waits for all copies.
// Waits are bounded (FOTO_MOCK_TIMEOUT_S, default 60 s): a sequence mismatch -- the bug this
// transport exists to catch -- fails with ncclSystemError instead of hanging.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <utility>
#include <vector>

struct ncclComm {
    struct MockWorld* w;
    int rank;
};

namespace {

struct P2P {
    int src, dst;
    void* buf;
    size_t bytes;
    hipStream_t st;
    hipEvent_t ready;   // the issuing stream reached the operation
    bool matched = false;
    bool failed = false;
};

struct Gather {
    const void* send;
    void* recv;
    size_t bytes;
    hipStream_t st;
    hipEvent_t ready;
    hipEvent_t done = nullptr;
};

}  // namespace

struct MockWorld {
    int n = 0;
    std::mutex mu;
    std::condition_variable cv;
    std::map<std::pair<int, int>, std::deque<std::shared_ptr<P2P>>> sends, recvs;   // key (src, dst)
    std::vector<std::vector<std::shared_ptr<Gather>>> gathers;   // [rank][call index]
    std::vector<int> gathers_done;                               // completed collectives
    std::vector<hipEvent_t> events;                              // destroyed with the world
    int refs = 0;
    hipEvent_t event() {
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
        events.push_back(e);
        return e;
    }
};

namespace {

std::mutex g_mu;
std::map<std::string, MockWorld*> g_worlds;
unsigned long long g_ids = 0;

thread_local int t_depth = 0;
thread_local std::vector<std::shared_ptr<P2P>> t_pending;
thread_local ncclComm* t_comm = nullptr;

std::chrono::seconds timeout() {
    const char* e = getenv("FOTO_MOCK_TIMEOUT_S");
    return std::chrono::seconds(e ? std::max(1, atoi(e)) : 60);
}

// match queued pairs of one channel (caller holds w->mu)
bool match_channel(MockWorld* w, std::pair<int, int> key) {
    auto& sq = w->sends[key];
    auto& rq = w->recvs[key];
    while (!sq.empty() && !rq.empty()) {
        std::shared_ptr<P2P> s = sq.front(), r = rq.front();
        sq.pop_front();
        rq.pop_front();
        if (s->bytes != r->bytes) {   // NCCL would corrupt or hang: a test failure here
            s->failed = r->failed = true;
        } else {
            hipEvent_t copied = w->event();
            if (!copied || hipStreamWaitEvent(r->st, s->ready, 0) != hipSuccess ||
                hipMemcpyAsync(r->buf, s->buf, r->bytes, hipMemcpyDeviceToDevice, r->st) != hipSuccess ||
                hipEventRecord(copied, r->st) != hipSuccess || hipStreamWaitEvent(s->st, copied, 0) != hipSuccess)
                s->failed = r->failed = true;
        }
        s->matched = r->matched = true;
    }
    return true;
}

ncclResult_t post_group() {
    std::vector<std::shared_ptr<P2P>> ops;
    ops.swap(t_pending);
    if (ops.empty()) return ncclSuccess;
    MockWorld* w = t_comm->w;
    std::unique_lock<std::mutex> lk(w->mu);
    for (auto& op : ops) {
        op->ready = w->event();
        if (!op->ready || hipEventRecord(op->ready, op->st) != hipSuccess) return ncclUnhandledCudaError;
    }
    for (auto& op : ops) {
        const bool is_send = op->src == t_comm->rank;
        (is_send ? w->sends : w->recvs)[{op->src, op->dst}].push_back(op);
        match_channel(w, {op->src, op->dst});
    }
    w->cv.notify_all();
    const auto deadline = std::chrono::steady_clock::now() + timeout();
    auto all = [&] {
        for (auto& op : ops)
            if (!op->matched) return false;
        return true;
    };
    if (!w->cv.wait_until(lk, deadline, all)) return ncclSystemError;   // a peer never posted its half
    for (auto& op : ops)
        if (op->failed) return ncclInvalidUsage;
    return ncclSuccess;
}

}  // namespace

extern "C" {

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (mock)";
        case ncclSystemError: return "mock RCCL: timed out waiting for the peer's matching operation";
        case ncclInvalidUsage: return "mock RCCL: matched send / receive sizes differ";
        case ncclInvalidArgument: return "mock RCCL: invalid argument";
        case ncclInternalError: return "mock RCCL: communicator refused (FOTO_MOCK_FAIL_INIT)";
        default: return "mock RCCL: HIP error";
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    std::lock_guard<std::mutex> lk(g_mu);
    memset(id, 0, sizeof(*id));
    snprintf(id->internal, sizeof(id->internal), "foto-mock-rccl-%llu", ++g_ids);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    // FOTO_MOCK_FAIL_INIT=1: the communicator is refused (as real RCCL refuses two ranks on one
    // GPU) -- the failure path of bench.py's sharded headline (tests/test_gpu_bench.py)
    const char* fi = getenv("FOTO_MOCK_FAIL_INIT");
    if (fi && atoi(fi) != 0) return ncclInternalError;
    std::lock_guard<std::mutex> lk(g_mu);
    const std::string key(id.internal, strnlen(id.internal, sizeof(id.internal)));
    MockWorld*& w = g_worlds[key];
    if (!w) {
        w = new MockWorld();
        w->n = nranks;
        w->gathers.resize(nranks);
        w->gathers_done.assign(1, 0);
    }
    if (w->n != nranks) return ncclInvalidArgument;
    w->refs += 1;
    *comm = new ncclComm{w, rank};
    return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
    if (!comm || !count) return ncclInvalidArgument;
    *count = comm->w->n;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    if (!comm) return ncclInvalidArgument;
    std::lock_guard<std::mutex> lk(g_mu);
    MockWorld* w = comm->w;
    delete comm;
    if (--w->refs == 0) {
        (void)hipDeviceSynchronize();
        for (hipEvent_t e : w->events) (void)hipEventDestroy(e);
        for (auto it = g_worlds.begin(); it != g_worlds.end(); ++it)
            if (it->second == w) { g_worlds.erase(it); break; }
        delete w;
    }
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
    ++t_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_depth <= 0) return ncclInvalidUsage;
    if (--t_depth > 0) return ncclSuccess;
    return post_group();
}

static ncclResult_t p2p(bool send, const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                        hipStream_t st) {
    if (!comm || peer < 0 || peer >= comm->w->n || peer == comm->rank || type != ncclDouble) return ncclInvalidArgument;
    if (t_comm && t_comm != comm && !t_pending.empty()) return ncclInvalidUsage;   // one comm per group
    t_comm = comm;
    auto op = std::make_shared<P2P>();
    op->src = send ? comm->rank : peer;
    op->dst = send ? peer : comm->rank;
    op->buf = const_cast<void*>(buf);
    op->bytes = count * sizeof(double);
    op->st = st;
    t_pending.push_back(op);
    return t_depth > 0 ? ncclSuccess : post_group();
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    return p2p(true, buf, count, type, peer, comm, stream);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm, hipStream_t stream) {
    return p2p(false, buf, count, type, peer, comm, stream);
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t type, ncclComm_t comm,
                           hipStream_t st) {
    if (!comm || type != ncclDouble || t_depth > 0) return ncclInvalidArgument;
    MockWorld* w = comm->w;
    const size_t bytes = count * sizeof(double);
    // in place, as libfoto calls it: sendbuff is this rank's slot of recvbuff
    if ((const char*)sendbuff != (const char*)recvbuff + comm->rank * bytes) return ncclInvalidArgument;
    std::unique_lock<std::mutex> lk(w->mu);
    auto g = std::make_shared<Gather>();
    g->send = sendbuff;
    g->recv = recvbuff;
    g->bytes = bytes;
    g->st = st;
    g->ready = w->event();
    if (!g->ready || hipEventRecord(g->ready, st) != hipSuccess) return ncclUnhandledCudaError;
    auto& mine = w->gathers[comm->rank];
    const size_t k = mine.size();
    mine.push_back(g);
    if (w->gathers_done.size() <= k) w->gathers_done.resize(k + 1, 0);
    bool complete = true;
    for (int r = 0; r < w->n; ++r) complete = complete && w->gathers[r].size() > k;
    if (complete) {   // the last rank to arrive enqueues the collective on every rank's stream
        for (int r = 0; r < w->n; ++r) {
            Gather& R = *w->gathers[r][k];
            for (int h = 0; h < w->n; ++h) {
                if (h == r) continue;
                Gather& H = *w->gathers[h][k];
                if (H.bytes != R.bytes) return ncclInvalidUsage;
                if (hipStreamWaitEvent(R.st, H.ready, 0) != hipSuccess ||
                    hipMemcpyAsync((char*)R.recv + h * R.bytes, H.send, R.bytes, hipMemcpyDeviceToDevice, R.st) !=
                        hipSuccess)
                    return ncclUnhandledCudaError;
            }
            R.done = w->event();
            if (!R.done || hipEventRecord(R.done, R.st) != hipSuccess) return ncclUnhandledCudaError;
        }
        for (int h = 0; h < w->n; ++h)   // a rank's slot is rewritten later: wait for every reader
            for (int r = 0; r < w->n; ++r)
                if (r != h && hipStreamWaitEvent(w->gathers[h][k]->st, w->gathers[r][k]->done, 0) != hipSuccess)
                    return ncclUnhandledCudaError;
        w->gathers_done[k] = 1;
        w->cv.notify_all();
        return ncclSuccess;
    }
    const auto deadline = std::chrono::steady_clock::now() + timeout();
    if (!w->cv.wait_until(lk, deadline, [&] { return w->gathers_done[k] != 0; })) return ncclSystemError;
    return ncclSuccess;
}

}  // extern "C"
