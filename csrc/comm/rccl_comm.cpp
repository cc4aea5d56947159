// Native RCCL communicator on a dedicated HIP stream (SURVEY.md §1 L1', N16).
//
// The reference has no collective code at all (its only NCCL touchpoint is a transitive lock entry,
// /root/reference/poetry.lock:1222); this is the framework's own comm layer for data parallelism
// over xGMI.  One process per GPU; the communicator is created from an ncclUniqueId that rank 0
// draws and the Python side exchanges over the torch.distributed rendezvous
// (replicann_amd/parallel/comm.py).  Design points:
//
//  * every collective runs on ONE high-priority comm stream owned by the communicator.  It is
//    forked from the caller's (compute) stream with an event, so it starts after the kernels that
//    produced the bucket and overlaps whatever the compute stream does next (the rest of the
//    backward); comm_wait() joins it back (stream-ordered, no host synchronisation);
//  * fork/join are plain event record/wait pairs, so a step that issues collectives can be
//    captured into a hipGraph: the comm stream joins the capture and the RCCL kernels become
//    graph nodes (ordered exactly as issued);
//  * failure detection: a watchdog thread per communicator polls the last collective's done
//    event; if it has not completed within the timeout, or RCCL reports an asynchronous error,
//    the communicator is aborted (ncclCommAbort unblocks every pending RCCL kernel) and the next
//    call raises, naming the collective that hung.
//
//  * proxy mode (comm_init_proxy): no RCCL communicator; every collective launches the comm-proxy
//    kernel (csrc/kernels/comm_proxy.hip) on the same comm stream with the same fork/join, moving
//    the emulated W-rank ring's per-GPU volume at an xGMI-like rate — the one-GPU stand-in that
//    makes the backward's GEMM ↔ collective interference measurable (bench.py --comm proxy).
//
// Handles are small integers into a process-wide table so they pass through TORCH_LIBRARY schemas.

#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <torch/library.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

extern "C" void rn_comm_proxy(void* buf, long bytes, double volume_bytes, int wgs, double gbps, hipStream_t st);
extern "C" void rn_cast_f32_bf16(const float* in, void* out, long n, hipStream_t st);

namespace {

using at::Tensor;

#define RCCL_CHECK(expr)                                                                      \
    do {                                                                                      \
        ncclResult_t _r = (expr);                                                             \
        TORCH_CHECK(_r == ncclSuccess, "RCCL error ", int(_r), " (", ncclGetErrorString(_r), \
                    ") in " #expr);                                                           \
    } while (0)
#define HIP_OK(expr)                                                                               \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        TORCH_CHECK(_e == hipSuccess, "HIP error ", hipGetErrorString(_e), " in " #expr);          \
    } while (0)

struct Comm {
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1, device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t fork = nullptr;  // recorded on the caller's stream, waited by the comm stream
    hipEvent_t done = nullptr;        // recorded on the comm stream after every collective (capture-safe join)
    hipEvent_t done_eager = nullptr;  // recorded after EAGER collectives only (never inside a capture)
    // watchdog state: one pooled event per outstanding eager collective, oldest first
    std::mutex mu;
    std::condition_variable cv;
    std::thread watchdog;
    bool stop = false;
    struct Pending {
        hipEvent_t ev;
        std::chrono::steady_clock::time_point issued;
        std::string op;
    };
    std::deque<Pending> pending;
    std::vector<hipEvent_t> free_events;
    double timeout_s = 600.0;
    std::atomic<int> failed{0};  // 0 ok, 1 timed out, 2 async RCCL error
    std::string failure;
    int64_t n_collectives = 0;
    int64_t bytes = 0;
    // proxy mode: emulated world size, workgroups, per-GPU bus bandwidth (GB/s)
    bool proxy = false;
    int proxy_world = 8, proxy_wgs = 32;
    double proxy_gbps = 300.0;

    void stop_watchdog() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        if (watchdog.joinable()) watchdog.join();
    }
    // at process exit (static destruction) only the thread is stopped: the HIP runtime and the
    // peers may already be gone, so no stream/communicator teardown happens here
    ~Comm() { stop_watchdog(); }
    hipEvent_t take_event() {  // under mu
        if (!free_events.empty()) {
            hipEvent_t e = free_events.back();
            free_events.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
        return e;
    }
};

std::mutex g_mu;
std::vector<std::unique_ptr<Comm>> g_comms;

Comm& get(int64_t h) {
    std::lock_guard<std::mutex> lk(g_mu);
    TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h], "invalid replicann comm handle ", h);
    return *g_comms[h];
}

void check_alive(Comm& c) {
    if (c.failed.load()) {
        std::lock_guard<std::mutex> lk(c.mu);
        TORCH_CHECK(false, "replicann comm (rank ", c.rank, "/", c.world, ") aborted: ", c.failure);
    }
}

void watchdog_loop(Comm* c) {
    // relaxed capture interaction: this thread's event queries must never invalidate a hipGraph
    // capture that the training thread runs meanwhile (PyTorch captures in global mode)
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    hipThreadExchangeStreamCaptureMode(&mode);
    std::unique_lock<std::mutex> lk(c->mu);
    while (!c->stop) {
        c->cv.wait_for(lk, std::chrono::milliseconds(100));
        if (c->stop || c->failed.load()) continue;
        ncclResult_t async = ncclSuccess;
        if (c->comm && ncclCommGetAsyncError(c->comm, &async) == ncclSuccess && async != ncclSuccess &&
            async != ncclInProgress) {
            c->failure = std::string("asynchronous RCCL error: ") + ncclGetErrorString(async);
            c->failed = 2;
            ncclCommAbort(c->comm);
            continue;
        }
        if (c->pending.empty()) continue;
        hipSetDevice(c->device);
        // retire finished collectives in issue order; the timeout runs from the OLDEST unfinished
        while (!c->pending.empty() && hipEventQuery(c->pending.front().ev) == hipSuccess) {
            c->free_events.push_back(c->pending.front().ev);
            c->pending.pop_front();
        }
        if (c->pending.empty()) continue;
        const auto& old = c->pending.front();
        double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - old.issued).count();
        if (waited > c->timeout_s) {
            c->failure = "collective '" + old.op + "' did not complete within " + std::to_string(c->timeout_s) +
                         " s (a peer rank is missing or hung)";
            c->failed = 1;
            if (c->comm) ncclCommAbort(c->comm);
        }
    }
}

ncclDataType_t nccl_dtype(const Tensor& t) {
    switch (t.scalar_type()) {
        case at::kFloat: return ncclFloat32;
        case at::kBFloat16: return ncclBfloat16;
        case at::kHalf: return ncclFloat16;
        case at::kDouble: return ncclFloat64;
        case at::kInt: return ncclInt32;
        case at::kLong: return ncclInt64;
        case at::kByte: return ncclUint8;
        default: TORCH_CHECK(false, "replicann comm: unsupported dtype ", t.scalar_type());
    }
}

ncclRedOp_t nccl_op(int64_t op) {
    switch (op) {
        case 0: return ncclSum;
        case 1: return ncclMax;
        case 2: return ncclMin;
        case 3: return ncclAvg;
        default: TORCH_CHECK(false, "replicann comm: unknown reduction ", op);
    }
}

// fork the comm stream off the caller's stream; returns whether the caller is capturing
bool fork_from_current(Comm& c) {
    hipStream_t cs = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(c.device).stream();
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    HIP_OK(hipStreamIsCapturing(cs, &st));
    bool cap = st == hipStreamCaptureStatusActive;  // captured collectives are not watched
    HIP_OK(hipEventRecord(c.fork, cs));
    HIP_OK(hipStreamWaitEvent(c.stream, c.fork, 0));
    return cap;
}

void after_issue(Comm& c, bool capturing, const char* what, int64_t nbytes) {
    HIP_OK(hipEventRecord(c.done, c.stream));
    c.n_collectives += 1;
    c.bytes += nbytes;
    if (!capturing) {
        HIP_OK(hipEventRecord(c.done_eager, c.stream));
        std::lock_guard<std::mutex> lk(c.mu);
        hipEvent_t e = c.take_event();
        HIP_OK(hipEventRecord(e, c.stream));
        c.pending.push_back({e, std::chrono::steady_clock::now(), what});
    }
}

// proxy mode: the emulated collective's per-GPU volume through the proxy kernel
void proxy_issue(Comm& c, const Tensor& t, double volume) {
    rn_comm_proxy(t.data_ptr(), t.numel() * t.element_size(), volume, c.proxy_wgs, c.proxy_gbps, c.stream);
}

// ---------------------------------------------------------------- ops

Tensor comm_unique_id() {
    ncclUniqueId id;
    RCCL_CHECK(ncclGetUniqueId(&id));
    Tensor out = at::empty({NCCL_UNIQUE_ID_BYTES}, at::TensorOptions().dtype(at::kByte));
    std::memcpy(out.data_ptr(), id.internal, NCCL_UNIQUE_ID_BYTES);
    return out;
}

int64_t comm_init(const Tensor& uid, int64_t rank, int64_t world, int64_t device, double timeout_s) {
    TORCH_CHECK(uid.device().is_cpu() && uid.scalar_type() == at::kByte && uid.numel() == NCCL_UNIQUE_ID_BYTES,
                "comm_init: uid must be the 128-byte CPU uint8 tensor from comm_unique_id()");
    TORCH_CHECK(rank >= 0 && rank < world, "comm_init: rank ", rank, " outside world ", world);
    ncclUniqueId id;
    std::memcpy(id.internal, uid.contiguous().data_ptr(), NCCL_UNIQUE_ID_BYTES);
    auto c = std::make_unique<Comm>();
    c->rank = (int)rank;
    c->world = (int)world;
    c->device = (int)device;
    c->timeout_s = timeout_s;
    c10::hip::HIPGuardMasqueradingAsCUDA guard(at::Device(at::kCUDA, (int)device));
    int lo = 0, hi = 0;
    HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    // hi = greatest priority: collectives' workgroups dispatch ahead of queued compute work
    HIP_OK(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi));
    HIP_OK(hipEventCreateWithFlags(&c->fork, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&c->done_eager, hipEventDisableTiming));
    RCCL_CHECK(ncclCommInitRank(&c->comm, (int)world, id, (int)rank));
    c->watchdog = std::thread(watchdog_loop, c.get());
    std::lock_guard<std::mutex> lk(g_mu);
    g_comms.push_back(std::move(c));
    return (int64_t)g_comms.size() - 1;
}

int64_t comm_init_proxy(int64_t device, int64_t world, int64_t wgs, double gbps, double timeout_s) {
    TORCH_CHECK(world >= 1 && wgs >= 1 && gbps > 0, "comm_init_proxy: world >= 1, wgs >= 1, gbps > 0");
    auto c = std::make_unique<Comm>();
    c->rank = 0;
    c->world = 1;  // the process group is one rank; proxy_world is what the volume emulates
    c->device = (int)device;
    c->timeout_s = timeout_s;
    c->proxy = true;
    c->proxy_world = (int)world;
    c->proxy_wgs = (int)wgs;
    c->proxy_gbps = gbps;
    c10::hip::HIPGuardMasqueradingAsCUDA guard(at::Device(at::kCUDA, (int)device));
    int lo = 0, hi = 0;
    HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_OK(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi));
    HIP_OK(hipEventCreateWithFlags(&c->fork, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&c->done_eager, hipEventDisableTiming));
    c->watchdog = std::thread(watchdog_loop, c.get());
    std::lock_guard<std::mutex> lk(g_mu);
    g_comms.push_back(std::move(c));
    return (int64_t)g_comms.size() - 1;
}

void comm_all_reduce(int64_t h, Tensor t, int64_t op) {
    Comm& c = get(h);
    check_alive(c);
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "comm_all_reduce: needs a contiguous GPU tensor");
    TORCH_CHECK(t.device().index() == c.device, "comm_all_reduce: tensor on cuda:", t.device().index(),
                ", communicator on cuda:", c.device);
    c10::hip::HIPGuardMasqueradingAsCUDA guard(t.device());
    bool cap = fork_from_current(c);
    if (c.proxy) {  // ring all-reduce: reduce-scatter + all-gather, each (W-1)/W of the buffer
        const double S = (double)t.numel() * t.element_size();
        proxy_issue(c, t, 2.0 * (c.proxy_world - 1) / c.proxy_world * S);
    } else
        RCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), nccl_dtype(t), nccl_op(op), c.comm,
                                 c.stream));
    after_issue(c, cap, "all_reduce", t.numel() * t.element_size());
}

void comm_broadcast(int64_t h, Tensor t, int64_t root) {
    Comm& c = get(h);
    check_alive(c);
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "comm_broadcast: needs a contiguous GPU tensor");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(t.device());
    bool cap = fork_from_current(c);
    if (c.proxy) proxy_issue(c, t, (double)t.numel() * t.element_size());
    else
        RCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), nccl_dtype(t), (int)root, c.comm,
                                 c.stream));
    after_issue(c, cap, "broadcast", t.numel() * t.element_size());
}

// out (world x in.numel) <- every rank's `in`, in rank order
void comm_all_gather(int64_t h, const Tensor& in, Tensor out) {
    Comm& c = get(h);
    check_alive(c);
    TORCH_CHECK(in.is_cuda() && in.is_contiguous() && out.is_contiguous() && out.numel() == in.numel() * c.world &&
                    out.scalar_type() == in.scalar_type(),
                "comm_all_gather: out must hold world x in.numel() elements of in's dtype");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(in.device());
    // proxy, world 1: the result is the input, copied on the caller's stream before the fork
    if (c.proxy) out.copy_(in.reshape(out.sizes()));
    bool cap = fork_from_current(c);
    if (c.proxy) {
        // a W-rank ring all-gather moves (W-1)/W of the full output per GPU (world 1: out is that output)
        proxy_issue(c, out, (double)(c.proxy_world - 1) / c.proxy_world * out.numel() * out.element_size());
    } else
        RCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), nccl_dtype(in), c.comm, c.stream));
    after_issue(c, cap, "all_gather", out.numel() * out.element_size());
}

// out (in.numel / world) <- this rank's reduced shard of `in`
void comm_reduce_scatter(int64_t h, const Tensor& in, Tensor out, int64_t op) {
    Comm& c = get(h);
    check_alive(c);
    TORCH_CHECK(in.is_cuda() && in.is_contiguous() && out.is_contiguous() && in.numel() == out.numel() * c.world &&
                    out.scalar_type() == in.scalar_type(),
                "comm_reduce_scatter: in must hold world x out.numel() elements of out's dtype");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(in.device());
    // proxy, world 1: the result is the input, copied on the caller's stream before the fork
    if (c.proxy) out.copy_(in.reshape(out.sizes()));
    bool cap = fork_from_current(c);
    if (c.proxy) {
        // a W-rank ring reduce-scatter moves (W-1)/W of the full input per GPU (world 1: out = in)
        proxy_issue(c, out, (double)(c.proxy_world - 1) / c.proxy_world * out.numel() * out.element_size());
    } else
        RCCL_CHECK(ncclReduceScatter(in.data_ptr(), out.data_ptr(), (size_t)out.numel(), nccl_dtype(in), nccl_op(op),
                                     c.comm, c.stream));
    after_issue(c, cap, "reduce_scatter", in.numel() * in.element_size());
}

// The second half of the reducer's reduce-scatter -> all-gather path, on the comm stream right after
// the reduce-scatter that filled shard32: narrow this rank's reduced fp32 shard to bf16 (shard16), then
// all-gather the bf16 shards into `full` (rank order).  bf16 is rounded ONCE, after the exact fp32
// cross-rank sum, and the gather moves half the bytes of an fp32 all-gather.
void comm_narrow_all_gather(int64_t h, const Tensor& shard32, Tensor shard16, Tensor full) {
    Comm& c = get(h);
    check_alive(c);
    TORCH_CHECK(shard32.is_cuda() && shard32.is_contiguous() && shard32.scalar_type() == at::kFloat &&
                    shard16.is_contiguous() && shard16.scalar_type() == at::kBFloat16 &&
                    shard16.numel() == shard32.numel() && full.is_contiguous() &&
                    full.scalar_type() == at::kBFloat16 && full.numel() == shard16.numel() * c.world,
                "comm_narrow_all_gather: fp32 shard, bf16 shard of the same size, bf16 full = world x shard");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(shard32.device());
    bool cap = fork_from_current(c);
    rn_cast_f32_bf16(shard32.data_ptr<float>(), shard16.data_ptr(), shard32.numel(), c.stream);
    if (c.proxy) {
        // world 1: the gathered result is the narrowed shard itself
        HIP_OK(hipMemcpyAsync(full.data_ptr(), shard16.data_ptr(), shard16.numel() * 2, hipMemcpyDeviceToDevice, c.stream));
        proxy_issue(c, full, (double)(c.proxy_world - 1) / c.proxy_world * full.numel() * full.element_size());
    } else
        RCCL_CHECK(ncclAllGather(shard16.data_ptr(), full.data_ptr(), (size_t)shard16.numel(), ncclBfloat16, c.comm,
                                 c.stream));
    after_issue(c, cap, "all_gather", full.numel() * full.element_size());
}

// the caller's current stream waits for every collective issued so far (no host sync)
void comm_wait(int64_t h) {
    Comm& c = get(h);
    check_alive(c);
    c10::hip::HIPGuardMasqueradingAsCUDA guard(at::Device(at::kCUDA, c.device));
    hipStream_t cs = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(c.device).stream();
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    HIP_OK(hipStreamIsCapturing(cs, &st));
    // inside a capture: join the collectives recorded in it; eager: the last eager collective
    // (an event last recorded inside a finished capture must not be waited on eagerly)
    HIP_OK(hipStreamWaitEvent(cs, st == hipStreamCaptureStatusActive ? c.done : c.done_eager, 0));
}

// host blocks until every issued collective finished (raises if the communicator was aborted)
void comm_synchronize(int64_t h) {
    Comm& c = get(h);
    c10::hip::HIPGuardMasqueradingAsCUDA guard(at::Device(at::kCUDA, c.device));
    while (hipEventQuery(c.done_eager) == hipErrorNotReady) {
        check_alive(c);
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    check_alive(c);
}

// [rank, world, collectives issued, bytes issued, failed]
std::vector<int64_t> comm_info(int64_t h) {
    Comm& c = get(h);
    return {c.rank, c.world, c.n_collectives, c.bytes, (int64_t)c.failed.load()};
}

// stop the watchdog thread only (interpreter exit: no HIP call may race the runtime's teardown)
void comm_quiesce(int64_t h) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (h >= 0 && h < (int64_t)g_comms.size() && g_comms[h]) g_comms[h]->stop_watchdog();
}

void comm_destroy(int64_t h) {
    std::unique_ptr<Comm> c;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h], "invalid replicann comm handle ", h);
        c = std::move(g_comms[h]);
    }
    c->stop_watchdog();
    c10::hip::HIPGuardMasqueradingAsCUDA guard(at::Device(at::kCUDA, c->device));
    if (c->failed.load() == 0) {
        hipStreamSynchronize(c->stream);
        if (c->comm) ncclCommDestroy(c->comm);
    }
    hipEventDestroy(c->fork);
    hipEventDestroy(c->done);
    hipEventDestroy(c->done_eager);
    for (auto& p : c->pending) hipEventDestroy(p.ev);
    for (auto e : c->free_events) hipEventDestroy(e);
    hipStreamDestroy(c->stream);
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(replicann, m) {
    m.def("comm_unique_id() -> Tensor", &comm_unique_id);
    m.def("comm_init(Tensor uid, int rank, int world, int device, float timeout_s) -> int", &comm_init);
    m.def("comm_init_proxy(int device, int world, int wgs, float gbps, float timeout_s) -> int", &comm_init_proxy);
    m.def("comm_all_reduce(int h, Tensor(a!) t, int op) -> ()", &comm_all_reduce);
    m.def("comm_broadcast(int h, Tensor(a!) t, int root) -> ()", &comm_broadcast);
    m.def("comm_all_gather(int h, Tensor inp, Tensor(a!) out) -> ()", &comm_all_gather);
    m.def("comm_reduce_scatter(int h, Tensor inp, Tensor(a!) out, int op) -> ()", &comm_reduce_scatter);
    m.def("comm_narrow_all_gather(int h, Tensor shard32, Tensor(a!) shard16, Tensor(b!) full) -> ()",
          &comm_narrow_all_gather);
    m.def("comm_wait(int h) -> ()", &comm_wait);
    m.def("comm_synchronize(int h) -> ()", &comm_synchronize);
    m.def("comm_info(int h) -> int[]", &comm_info);
    m.def("comm_quiesce(int h) -> ()", &comm_quiesce);
    m.def("comm_destroy(int h) -> ()", &comm_destroy);
}
