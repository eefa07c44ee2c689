// loopback_backend.cc — see loopback_backend.h.
#include "loopback_backend.h"

#include <hip/hip_runtime_api.h>
#include <time.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <vector>
#include <cstdio>
#include <memory>
#include <string>

#include "context.h"
#include "hip_exponent_quantizer_ppp.h"
#include "prepostprocessor.h"
#include "switchml_hip.h"
#include "xgmi_switch.h"

namespace switchml {

namespace {

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw SwitchMLFatal(std::string(what) + ": " + hipGetErrorString(e));
}

void sml_ok(int s, const char* what) {
    if (s != SML_OK)
        throw SwitchMLFatal(std::string(what) + ": " + sml_status_string((sml_status_t)s) + " " + sml_last_error());
}

// Wait for the worker's stream: poll for a short while (a slice's kernels
// usually finish within it), then block in hipStreamSynchronize.
void stream_wait(hipStream_t st) {
    const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(SpinMicros());
    do {
        const hipError_t q = hipStreamQuery(st);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) hip_ok(q, "hipStreamQuery");
    } while (std::chrono::steady_clock::now() < until);
    hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
}

// Grow-only device buffer owned by one worker thread, used only on that
// worker's stream.  Stream-ordered (hipFreeAsync / hipMallocAsync on the
// stream): the old buffer is released after the work already queued on it,
// and no device-wide synchronisation happens on the worker thread — hipFree
// waits for every stream of the device, which a worker serving RCCL's
// CollNet proxy must not do while RCCL's kernels wait on that proxy.
struct DeviceBuffer {
    void* p = nullptr;
    size_t cap = 0;
    hipStream_t owner = nullptr;
    void Abandon() { p = nullptr; cap = 0; }   // the owner stream is wedged: leak, never free
    void* get(size_t bytes, hipStream_t st) {
        if (bytes > cap) {
            if (p) hip_ok(hipFreeAsync(p, owner), "hipFreeAsync");
            p = nullptr;
            cap = std::max<size_t>(bytes, 4096);
            hip_ok(hipMallocAsync(&p, cap, st), "hipMallocAsync");
            owner = st;
        }
        return p;
    }
    ~DeviceBuffer() {
        if (p) (void)hipFreeAsync(p, owner);
    }
};

// Grow-only host buffer: page-locked (hipHostMalloc) or pageable (malloc).
struct HostBuffer {
    void* p = nullptr;
    size_t cap = 0;
    bool pinned = false;
    void* get(size_t bytes, bool pin) {
        if (bytes > cap || pin != pinned) {
            release();
            cap = std::max<size_t>(bytes, 4096);
            pinned = pin;
            if (pin) hip_ok(hipHostMalloc(&p, cap, hipHostMallocDefault), "hipHostMalloc");
            else if (!(p = std::malloc(cap))) throw SwitchMLFatal("malloc failed");
        }
        return p;
    }
    void release() {
        if (!p) return;
        if (pinned) (void)hipHostFree(p);
        else std::free(p);
        p = nullptr;
        cap = 0;
    }
    ~HostBuffer() { release(); }
};

struct WorkerState {
    DeviceBuffer in, out, payload, exps, ring, ring_extra;
    HostBuffer hring, hring_extra;
    // the worker's stream is wedged (XgmiSwitch::Wedged): its unfinished work
    // may still use these buffers, so they are leaked, not freed
    void Abandon() {
        for (DeviceBuffer* b : {&in, &out, &payload, &exps, &ring, &ring_extra}) b->Abandon();
        hring.p = hring_extra.p = nullptr;
        hring.cap = hring_extra.cap = 0;
    }
};

// DummyWorkerThread's per-packet loop (dummy_worker_thread.cc:86-177) with
// in-order delivery over a device-resident ring of b packets.
void run_packet_loop(HipExponentQuantizerPPP& ppp, const Config& cfg, WorkerState& ws, bool extra_batch) {
    const uint64_t P = ppp.ltu_numel();
    const uint64_t B = ppp.total_main_num_ltus();
    const uint64_t b = ppp.batch_num_ltus();
    const uint64_t total = B + (extra_batch ? b : 0);
    const std::string& where = cfg.backend_.hip.packet_ring;
    int32_t* ring;
    uint8_t* extra;
    if (where == "device") {
        ring = static_cast<int32_t*>(ws.ring.get(b * P * 4, ppp.stream()));
        extra = static_cast<uint8_t*>(ws.ring_extra.get(b * 2, ppp.stream()));
        hip_ok(hipMemsetAsync(ring, 0, b * P * 4, ppp.stream()), "hipMemsetAsync");
    } else {
        const bool pin = where == "pinned";
        ring = static_cast<int32_t*>(ws.hring.get(b * P * 4, pin));
        extra = static_cast<uint8_t*>(ws.hring_extra.get(b * 2, pin));
        std::memset(ring, 0, b * P * 4);
    }
    // ProcessPacket (every entry of the packet x W, dummy_backend.cc:72-84) on
    // the device for a device-addressable ring (HBM or pinned host memory, in
    // the same launch as the PPP's calls), on the CPU for a pageable one.
    //
    // The reference handles one packet per loop trip: packet p comes back,
    // ProcessPacket, PostprocessSingle(p), PreprocessSingle(p + b) into the
    // same ring slot.  Slots are independent, so the packets of one pass over
    // the ring (slots s0 .. s0 + w - 1, w <= b) go as one burst — the way a
    // DPDK worker handles an rx burst and refills its mbufs — with the same
    // calls per slot in the same order: PostprocessReuseBurst (post of p, pre
    // of p + b into the slot).  A device-addressable ring runs the whole trip,
    // ProcessPacket included, as ONE launch per pass; the HBM ring stays
    // stream-ordered (no host sync), a host ring completes each burst before
    // the call returns (the packets would go to the NIC next).
    const uint16_t W = cfg.general_.num_workers;
    const bool dev_ring = where == "device";
    const bool proc = cfg.backend_.dummy.process_packets;
    ppp.SetStreamOrdered(dev_ring);
    std::vector<uint64_t> ids(b);
    std::vector<void*> ents(b), exs(b);
    for (uint64_t p = 0; p < b; p++) {
        ids[p] = p;
        ents[p] = ring + p * P;
        exs[p] = extra + p * 2;
    }
    ppp.PreprocessBurst((uint32_t)b, ids.data(), ents.data(), exs.data());
    for (uint64_t p0 = 0; p0 < total; p0 += b) {
        const uint64_t w = std::min<uint64_t>(b, total - p0);   // p0 % b == 0: slots 0 .. w - 1
        for (uint64_t s = 0; s < w; s++) ids[s] = p0 + s;
        if (proc && where != "pageable") {
            ppp.ProcessPostprocessReuseBurst((uint32_t)w, ids.data(), ents.data(), exs.data());
            continue;
        }
        if (proc)
            for (uint64_t i = 0; i < w * P; i++)
                ring[i] = (int32_t)__builtin_bswap32(__builtin_bswap32((uint32_t)ring[i]) * (uint32_t)W);
        ppp.PostprocessReuseBurst((uint32_t)w, ids.data(), ents.data(), exs.data(), b, total);
    }
    ppp.SetStreamOrdered(false);
}

uint64_t run_slice(PrePostProcessor& base, const Config& cfg, WorkerState& ws, JobSlice& js, XgmiSwitch* xs,
                   WorkerTid tid) {
    auto* ppp = dynamic_cast<HipExponentQuantizerPPP*>(&base);
    if (!ppp) {  // bypass: count packets, move nothing (bypass_ppp.h)
        const uint64_t B = base.SetupJobSlice(&js);
        base.CleanupJobSlice();
        return B;
    }
    hipStream_t st = ppp->stream();
    Tensor& t = js.slice;
    const size_t bytes = t.numel * DataTypeSize(t.data_type);
    // Device tensors are used in place; pinned host tensors too, through
    // their device mapping (the kernels read and write them over PCIe, both
    // directions at once — "zero-copy"); pageable host tensors are
    // staged through HBM with copies on the worker's stream.
    void* in_d = DeviceAddress(t.in_ptr);
    // the in-node switch reads its input twice (exponents, then quantize):
    // a host input is copied into HBM once instead of crossing PCIe twice
    if (xs && in_d && !IsDevicePointer(t.in_ptr)) in_d = nullptr;
    void* out_d = DeviceAddress(t.out_ptr);

    JobSlice staged = js;
    if (in_d) {
        staged.slice.in_ptr = in_d;
    } else {
        staged.slice.in_ptr = ws.in.get(bytes, st);
        hip_ok(hipMemcpyAsync(staged.slice.in_ptr, t.in_ptr, bytes, hipMemcpyHostToDevice, st), "hipMemcpyAsync H2D");
    }
    if (out_d) staged.slice.out_ptr = out_d;
    else staged.slice.out_ptr = (t.out_ptr == t.in_ptr) ? staged.slice.in_ptr : ws.out.get(bytes, st);

    const uint64_t B = ppp->SetupJobSlice(&staged);
    const uint64_t P = ppp->ltu_numel();
    const uint16_t W = cfg.general_.num_workers;
    const std::string& mode = cfg.backend_.hip.mode;
    const bool is_float = t.data_type == FLOAT32;
    uint64_t packets = B + (ppp->NeedsExtraBatch() ? ppp->batch_num_ltus() : 0);

    if (xs) {
        // the in-node switch: this slice across the W workers (synchronous)
        xs->AllReduceSlice(tid, staged.slice.in_ptr, staged.slice.out_ptr, t.numel, t.data_type, st);
    } else if (mode == "packet") {
        run_packet_loop(*ppp, cfg, ws, ppp->NeedsExtraBatch());
    } else if (mode == "fused" && is_float && cfg.backend_.dummy.process_packets) {
        sml_ok(sml_roundtrip_loopback(static_cast<const float*>(staged.slice.in_ptr),
                                      static_cast<float*>(staged.slice.out_ptr), t.numel, (uint32_t)P, W, nullptr,
                                      nullptr, cfg.backend_.hip.vcl ? SML_FLAG_ROUND_RNE : 0u, st),
               "sml_roundtrip_loopback");
    } else {  // bulk
        void* payload = ws.payload.get(B * P * 4, st);
        void* exps = ws.exps.get(B, st);
        ppp->PreprocessBulk(payload, exps, nullptr, false);
        if (cfg.backend_.dummy.process_packets)
            sml_ok(sml_loopback_aggregate(static_cast<int32_t*>(payload), B * P, W, 0, st), "sml_loopback_aggregate");
        ppp->PostprocessBulk(payload, exps, false);
    }
    if (!out_d)
        hip_ok(hipMemcpyAsync(t.out_ptr, staged.slice.out_ptr, bytes, hipMemcpyDeviceToHost, st), "hipMemcpyAsync D2H");
    // Everything is enqueued on the worker's stream (args captured at launch):
    // the caller records an event and retires the slice when it completes.
    ppp->CleanupJobSlice();
    return packets;
}

// Wait for an event: poll for a short while (a slice's kernels usually finish
// within it), then block.
void event_wait(hipEvent_t ev) {
    const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(SpinMicros());
    do {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) hip_ok(q, "hipEventQuery");
    } while (std::chrono::steady_clock::now() < until);
    hip_ok(hipEventSynchronize(ev), "hipEventSynchronize");
}

// The oldest in-flight slice's event, while no later job is queued yet: poll
// for either its completion or a new job (a framework posts its buckets one
// call at a time — blocking on the event would serialize the next job behind
// this one's kernels), for SpinMicros(); then block on the event.  True: the
// event completed (or failed: the caller's retire reports it); false: a job
// arrived first, go and overlap it.
template <class HasJob>
bool event_or_job(hipEvent_t ev, HasJob has_job) {
    const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(SpinMicros());
    do {
        if (hipEventQuery(ev) != hipErrorNotReady) return true;
        if (has_job()) return false;
    } while (std::chrono::steady_clock::now() < until);
    return true;
}

}  // namespace

void* DeviceAddress(void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) return p;
    if (a.type == hipMemoryTypeHost && a.devicePointer) return a.devicePointer;
    return nullptr;
}

bool IsHostMapped(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost && a.devicePointer;
}

bool IsDevicePointer(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

LoopbackBackend::LoopbackBackend(Context& context, Config& config) : context_(context), config_(config) {}

LoopbackBackend::~LoopbackBackend() { CleanupWorker(); }

void LoopbackBackend::SetupWorker() {
    if (config_.general_.backend == "xgmi" && !xgmi_) xgmi_.reset(new XgmiSwitch(config_, context_.device()));
    if (BatchEligible()) {
        threads_.emplace_back(&LoopbackBackend::BatchMain, this);
        return;
    }
    for (int i = 0; i < config_.general_.num_worker_threads; i++)
        threads_.emplace_back(&LoopbackBackend::WorkerMain, this, (WorkerTid)i);
}

bool LoopbackBackend::BatchEligible() const {
    const GeneralConfig& g = config_.general_;
    return config_.backend_.hip.batch_jobs > 0 && config_.backend_.hip.mode == "fused" && g.backend == "dummy" &&
           g.prepostprocessor != "bypass" && config_.backend_.dummy.process_packets &&
           config_.backend_.dummy.bandwidth <= 0;
}

// Batched dispatch.  The reference's worker threads each run their FIFO slice
// of every job (dummy_worker_thread.cc:73-177) because a CPU core is the unit
// of parallelism; on the GPU one launch already fills the chip, so here ONE
// thread takes the queued jobs whole and runs every slice of up to
// batch_jobs of them in one sml_roundtrip_loopback_batch launch — the same
// slice geometry (so the same bits) with one launch and one event per batch
// instead of num_worker_threads per job.  Jobs whose buffers overlap an
// earlier job of the batch start a new launch (stream order keeps them in
// FIFO order); INT32 and pageable-host jobs run slice by slice through
// run_slice on the same stream.  Completion of every slice is reported under
// its own worker thread id, so the scheduler, Stats and failure semantics are
// those of the threaded path.
void LoopbackBackend::BatchMain() {
    const GeneralConfig& g = config_.general_;
    const int T = g.num_worker_threads;
    std::shared_ptr<PrePostProcessor> ppp;
    try {
        hip_ok(hipSetDevice(context_.device()), "hipSetDevice");
        ppp = PrePostProcessor::CreateInstance(config_, 0, g.packet_numel * 4, g.max_outstanding_packets / T);
    } catch (const std::exception& e) {
        fprintf(stderr, "[switchml] batch worker: %s\n", e.what());
    }
    auto* hip_ppp = dynamic_cast<HipExponentQuantizerPPP*>(ppp.get());
    const uint64_t P = g.packet_numel;
    const uint64_t bmax = g.max_outstanding_packets / T;
    const size_t max_jobs = std::max<size_t>(1, std::min<size_t>(config_.backend_.hip.batch_jobs,
                                                                  SML_MAX_BATCH_SLICES / std::max(1, T)));
    const uint32_t coalesce_us = config_.backend_.hip.coalesce_us;
    const uint32_t rne = config_.backend_.hip.vcl ? SML_FLAG_ROUND_RNE : 0u;   // the VCL=1 build's rounding
    struct Piece {
        JobSlice js;
        WorkerTid tid;
        uint64_t packets;
        bool ok;
    };
    struct Batch {
        std::vector<Piece> pieces;
        hipEvent_t ev = nullptr;
    };
    constexpr size_t kMaxInFlight = 4;
    std::deque<Batch> inflight;
    std::vector<hipEvent_t> events;
    auto publish = [&](std::vector<Piece>& pieces, bool ok) {
        for (Piece& pc : pieces) {
            const bool good = ok && pc.ok;
            if (good) context_.GetStats().AddSlice(pc.tid, pc.packets, pc.js.slice.numel * DataTypeSize(pc.js.slice.data_type));
            context_.NotifyJobSliceCompletion(pc.tid, pc.js, good);
        }
    };
    auto retire = [&]() {
        Batch& b = inflight.front();
        bool ok = true;
        try {
            event_wait(b.ev);
        } catch (const std::exception& e) {
            fprintf(stderr, "[switchml] batch worker: %s\n", e.what());
            ok = false;
        }
        publish(b.pieces, ok);
        events.push_back(b.ev);
        inflight.pop_front();
    };
    WorkerState ws;
    std::vector<std::shared_ptr<Job>> jobs;
    uint64_t last_seq = 0;
    while (context_.GetContextState() == Context::RUNNING) {
        while (!inflight.empty() && hipEventQuery(inflight.front().ev) != hipErrorNotReady) retire();
        if (!inflight.empty() && (inflight.size() >= kMaxInFlight || !context_.HasJobAfter(last_seq))) {
            // nothing to overlap with: finish the oldest batch first.  (Unlike the
            // threaded path this does not poll for a new job meanwhile: jobs that
            // arrive while the batch runs join the next launch — for zero-copy
            // host buckets larger launches move more bytes per second over PCIe;
            // measured: configs[4] pinned 2.95 ms this way, 3.23 ms polling.)
            retire();
            continue;
        }
        jobs.clear();
        if (!context_.GetJobs(max_jobs, jobs)) continue;
        last_seq = jobs.back()->sched_seq.load(std::memory_order_relaxed);
        // Zero-copy host buckets: a framework posts its buckets one call at a
        // time, so the first one would otherwise go alone into a small launch;
        // PCIe moves 31 GB/s each way in a 26 MB launch but 37-42 in 100 MB+
        // ones (profiles/r02/zero_copy_probes.json).  While the next job
        // follows within coalesce_us of the last, it joins this launch.
        if (coalesce_us > 0 && jobs.size() < max_jobs) {
            bool host = false;
            for (const auto& j : jobs) host = host || (j->tensor_.numel > 0 && IsHostMapped(j->tensor_.in_ptr));
            auto last = std::chrono::steady_clock::now();
            while (host && jobs.size() < max_jobs && context_.GetContextState() == Context::RUNNING) {
                if (context_.HasJobAfter(last_seq)) {
                    if (!context_.GetJobs(max_jobs, jobs)) break;
                    last_seq = jobs.back()->sched_seq.load(std::memory_order_relaxed);
                    last = std::chrono::steady_clock::now();
                    continue;
                }
                if (std::chrono::steady_clock::now() - last > std::chrono::microseconds(coalesce_us)) break;
                std::this_thread::yield();
            }
        }

        // Every job taken here shares ONE completion event, recorded after
        // the last launch: jobs that must be split into several launches (a
        // buffer shared with an earlier job of the batch: stream order keeps
        // FIFO order) do not pay an event between kernels each.
        Batch cur;
        std::vector<sml_slice> segs;
        size_t seg_first = 0;                                   // first piece of the pending launch
        std::vector<std::pair<uintptr_t, uintptr_t>> reads, writes;   // kernel address ranges of the pending launch
        // Launch the pending slices (one sml_roundtrip_loopback_batch); a
        // failure fails exactly those slices.
        auto launch = [&]() {
            if (!segs.empty()) {
                try {
                    sml_ok(sml_roundtrip_loopback_batch(segs.data(), (uint32_t)segs.size(), (uint32_t)P,
                                                        g.num_workers, rne, hip_ppp->stream()),
                           "sml_roundtrip_loopback_batch");
                } catch (const std::exception& e) {
                    fprintf(stderr, "[switchml] batch worker: %s\n", e.what());
                    (void)hipStreamSynchronize(hip_ppp->stream());
                    for (size_t i = seg_first; i < cur.pieces.size(); i++) cur.pieces[i].ok = false;
                }
            }
            segs.clear();
            reads.clear();
            writes.clear();
            seg_first = cur.pieces.size();
        };
        auto overlaps = [](const std::vector<std::pair<uintptr_t, uintptr_t>>& v, uintptr_t a, uintptr_t b) {
            for (const auto& r : v)
                if (a < r.second && r.first < b) return true;
            return false;
        };
        for (auto& job : jobs) {
            const Tensor& t = job->tensor_;
            const size_t esz = DataTypeSize(t.data_type);
            const bool work = t.numel > 0 && !g.instant_job_completion && hip_ppp;
            void* in_d = work ? DeviceAddress(t.in_ptr) : nullptr;
            void* out_d = work ? DeviceAddress(t.out_ptr) : nullptr;
            const bool batched = work && t.data_type == FLOAT32 && in_d && out_d;
            if (batched) {
                const uintptr_t i0 = (uintptr_t)in_d, i1 = i0 + t.numel * esz;
                const uintptr_t o0 = (uintptr_t)out_d, o1 = o0 + t.numel * esz;
                if (overlaps(writes, i0, i1) || overlaps(writes, o0, o1) || overlaps(reads, o0, o1)) launch();
                reads.emplace_back(i0, i1);
                writes.emplace_back(o0, o1);
            } else if (work) {
                launch();   // keep FIFO order on the stream
            }
            for (int tid = 0; tid < T; tid++) {
                Piece pc{JobSlice(), (WorkerTid)tid, 0, true};
                pc.js.job = job;
                pc.js.slice = t;
                Numel off, n;
                FifoSliceGeometry(t.numel, T, tid, &off, &n);
                pc.js.slice.numel = n;
                pc.js.slice.OffsetPtrs(off);
                if (!work || n == 0) {
                    pc.ok = work || t.numel == 0 || g.instant_job_completion;   // no pre/post-processor: failed
                } else if (tid == config_.backend_.dummy.fail_worker_thread) {
                    pc.ok = false;   // injected fault: this slice's buffers are not touched
                } else if (batched) {
                    const uint64_t B = n / P + (n % P != 0);
                    pc.packets = B + std::min<uint64_t>(B, bmax);
                    segs.push_back(sml_slice{static_cast<const float*>(in_d) + off, static_cast<float*>(out_d) + off, n});
                } else {
                    try {
                        pc.packets = run_slice(*ppp, config_, ws, pc.js, nullptr, (WorkerTid)tid);
                    } catch (const std::exception& e) {
                        fprintf(stderr, "[switchml] batch worker: job %llu failed: %s\n",
                                (unsigned long long)job->id_, e.what());
                        (void)hipStreamSynchronize(hip_ppp->stream());
                        pc.ok = false;
                    }
                }
                cur.pieces.push_back(std::move(pc));
            }
            if (!batched) seg_first = cur.pieces.size();   // its slices are not part of a pending launch
        }
        if (hip_ppp) launch();
        // one event for everything taken in this round
        try {
            if (!hip_ppp) throw SwitchMLFatal("no pre/post-processor");
            if (events.empty()) {
                hipEvent_t ev;
                hip_ok(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
                events.push_back(ev);
            }
            cur.ev = events.back();
            hip_ok(hipEventRecord(cur.ev, hip_ppp->stream()), "hipEventRecord");
            events.pop_back();
            inflight.push_back(std::move(cur));
        } catch (const std::exception& e) {
            fprintf(stderr, "[switchml] batch worker: %s\n", e.what());
            if (hip_ppp) (void)hipStreamSynchronize(hip_ppp->stream());   // nothing may still touch the buffers
            while (!inflight.empty()) retire();
            publish(cur.pieces, false);
        }
    }
    // stopping: batches in flight own their buffers until their kernels finish
    while (!inflight.empty()) retire();
    for (hipEvent_t ev : events) (void)hipEventDestroy(ev);
}

void LoopbackBackend::CleanupWorker() {
    {
        std::lock_guard<std::mutex> lk(wire_mutex_);
    }
    wire_cv_.notify_all();
    for (auto& t : threads_)
        if (t.joinable()) t.join();
    threads_.clear();
    xgmi_.reset();   // leave the session (a barrier with the other workers)
}

void LoopbackBackend::WorkerMain(WorkerTid tid) {
    const GeneralConfig& g = config_.general_;
    const bool bypass = g.prepostprocessor == "bypass";
    std::shared_ptr<PrePostProcessor> ppp;
    std::string setup_error;
    try {
        if (!bypass) hip_ok(hipSetDevice(context_.device()), "hipSetDevice");
        // dummy_worker_thread.cc:59-62: ltu = packet_numel * 4 bytes, b_max = mop / T
        ppp = PrePostProcessor::CreateInstance(config_, tid, g.packet_numel * 4,
                                               g.max_outstanding_packets / g.num_worker_threads);
    } catch (const std::exception& e) {
        setup_error = e.what();
        fprintf(stderr, "[switchml] worker thread %d: %s\n", tid, e.what());
    }
    auto* hip_ppp = dynamic_cast<HipExponentQuantizerPPP*>(ppp.get());
    const float bw = config_.backend_.dummy.bandwidth;
    // Slices whose kernels are still running: the worker takes the next job's
    // slice (when one is queued) while the GPU finishes the previous one, and
    // publishes each slice's completion, in order, once its event has passed.
    // Up to kMaxInFlight per worker; the simulated wire (bandwidth > 0) keeps
    // the strict one-at-a-time loop of dummy_worker_thread.cc.
    constexpr size_t kMaxInFlight = 4;
    struct InFlight {
        JobSlice js;
        hipEvent_t ev;
        uint64_t packets;
    };
    std::deque<InFlight> inflight;
    std::vector<hipEvent_t> events;
    auto retire = [&](bool wait) {
        InFlight& f = inflight.front();
        bool ok = true;
        try {
            if (wait) event_wait(f.ev);
        } catch (const std::exception& e) {
            fprintf(stderr, "[switchml] worker thread %d: job %llu failed: %s\n", tid,
                    (unsigned long long)f.js.job->id_, e.what());
            ok = false;
        }
        if (ok) context_.GetStats().AddSlice(tid, f.packets, f.js.slice.numel * DataTypeSize(f.js.slice.data_type));
        context_.NotifyJobSliceCompletion(tid, f.js, ok);
        events.push_back(f.ev);
        inflight.pop_front();
    };
    WorkerState ws;
    JobSlice js;
    uint64_t last_seq = 0;  // sched_seq of the last job this thread took a slice of
    // this worker's stream did not finish within the in-node switch's bounded
    // wait: every later slice fails at once, nothing waits on the stream again
    bool wedged = false;
    const DummyBackendConfig& dummy = config_.backend_.dummy;
    while (context_.GetContextState() == Context::RUNNING) {
        while (!inflight.empty() && hipEventQuery(inflight.front().ev) != hipErrorNotReady) retire(true);
        if (!inflight.empty() && (inflight.size() >= kMaxInFlight || !context_.HasJobAfter(last_seq))) {
            // nothing to overlap with (yet): finish the oldest slice, unless a job arrives first
            if (inflight.size() >= kMaxInFlight ||
                event_or_job(inflight.front().ev, [&] { return context_.HasJobAfter(last_seq); }))
                retire(true);
            continue;
        }
        if (!context_.GetJobSlice(tid, js)) continue;
        last_seq = js.job->sched_seq.load(std::memory_order_relaxed);
        // empty slices and instant_job_completion never touch the PPP
        // (dummy_worker_thread.cc:87-93)
        const bool work = js.slice.numel > 0 && !g.instant_job_completion;
        bool ok = !work || ppp != nullptr;
        if (work && tid == config_.backend_.dummy.fail_worker_thread) {   // injected fault
            ok = false;
            // with the in-node switch the fault fails the exchange for every
            // worker (as a real mid-exchange failure does), not a barrier wait
            if (xgmi_) xgmi_->Poison();
        }
        if (work && wedged) ok = false;
        uint64_t packets = 0;
        if (ok && work) {
            try {
                if (hip_ppp && tid == dummy.stall_worker_thread && dummy.stall_ms > 0)   // injected stall
                    sml_ok(sml_debug_stall(dummy.stall_ms * 1000u, hip_ppp->stream()), "sml_debug_stall");
                packets = run_slice(*ppp, config_, ws, js, xgmi_.get(), tid);
                if (hip_ppp && bw <= 0) {
                    if (events.empty()) {
                        hipEvent_t ev;
                        hip_ok(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
                        events.push_back(ev);
                    }
                    hipEvent_t ev = events.back();
                    hip_ok(hipEventRecord(ev, hip_ppp->stream()), "hipEventRecord");
                    events.pop_back();
                    inflight.push_back(InFlight{js, ev, packets});
                    js = JobSlice();
                    continue;
                }
                if (hip_ppp) stream_wait(hip_ppp->stream());
            } catch (const std::exception& e) {
                fprintf(stderr, "[switchml] worker thread %d: job %llu failed: %s\n", tid,
                        (unsigned long long)js.job->id_, e.what());
                // nothing may still touch the buffers when the slice is
                // published FAILED.  With the in-node switch the wait is
                // bounded (backend.xgmi.timeout_ms): a device that does not
                // finish fails the slice now, and the worker, its stream and
                // buffers are abandoned rather than blocking here forever.
                if (hip_ppp && xgmi_) {
                    if (xgmi_->Wedged() || !xgmi_->WaitBounded(hip_ppp->stream())) {
                        wedged = true;
                        hip_ppp->Abandon();   // its stream stays alive: the switch's reaper waits on it
                        ws.Abandon();
                        xgmi_->NoteStuckStream(tid, hip_ppp->stream());
                    }
                } else if (hip_ppp) {
                    (void)hipStreamSynchronize(hip_ppp->stream());
                }
                ok = false;
            }
            if (ok && bw > 0) {  // the dummy backend's simulated wire time (dummy_backend.cc:124-133)
                const double ns = 1000.0 * (double)packets * g.packet_numel * 4 * 8 * g.num_worker_threads / bw;
                // interruptible: Stop() must not wait out a simulated wire
                std::unique_lock<std::mutex> lk(wire_mutex_);
                wire_cv_.wait_for(lk, std::chrono::nanoseconds((int64_t)std::min(ns, 9.0e18)),
                                  [this] { return context_.GetContextState() != Context::RUNNING; });
            }
            if (ok) context_.GetStats().AddSlice(tid, packets, js.slice.numel * DataTypeSize(js.slice.data_type));
        }
        context_.NotifyJobSliceCompletion(tid, js, ok);
        js = JobSlice();
    }
    // stopping: the in-flight slices still own their buffers until their
    // kernels finish; then they are published (FAILED: the context stopped)
    while (!inflight.empty()) retire(true);
    for (hipEvent_t ev : events) (void)hipEventDestroy(ev);
}

}  // namespace switchml
