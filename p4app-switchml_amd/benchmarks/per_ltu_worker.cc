// per_ltu_worker — a packet-driven worker exactly as the reference writes
// one: the PrePostProcessor comes from the factory by its config name
// (prepostprocessor.cc:32-41) and is called once per packet, in
// DummyWorkerThread's order (dummy_worker_thread.cc:106-163: Preprocess
// p in [0, b); then per returned packet p, PostprocessSingle(p) and
// PreprocessSingle(p + b) into the same ring slot) — the call pattern of
// DpdkWorkerThread's BuildPacket / ReusePacket (dpdk_worker_thread_utils.inc:134).
// The ring is pinned host memory (an mbuf pool stand-in); num_workers = 1, so
// the loopback's ProcessPacket is the identity.
//
// Usage: per_ltu_worker <prepostprocessor> <numel> <out.f32> [single | burst-registered]
//   input x[i] = float(i) * (-1)^i (allreduce_benchmark/main.cc:207-212) in HBM;
//   the dequantized output is written to <out.f32>.
//   single (default): one PreprocessSingle / PostprocessSingle per packet;
//   burst-registered: the same packet loop through the burst hooks
//   (PreprocessBurst, then PostprocessReuseBurst per ring pass), with the
//   ring and the extra-info slots in two separate hipHostRegister'd
//   allocations — a NIC pool whose device addresses need not equal its host
//   addresses, and whose extras are another registration.
// Exit 0: done; 3: per-packet calls refused (message on stdout) — at setup,
// before any packet, when the configured name takes only the bulk / burst
// hooks (PrePostProcessor::PerLtuCalls, what a packet-driven backend asks at
// configuration time), or by the PPP itself on the data path
// (PER_LTU_NO_SETUP_CHECK=1 skips the setup check); 1: any other failure.
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "config.h"
#include "job.h"
#include "prepostprocessor.h"

using namespace switchml;

static void ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw SwitchMLFatal(std::string(what) + ": " + hipGetErrorString(e));
}

int main(int argc, char** argv) {
    if (argc != 4 && argc != 5) {
        fprintf(stderr, "usage: %s <prepostprocessor> <numel> <out.f32> [single | burst-registered]\n", argv[0]);
        return 1;
    }
    const std::string mode = argc == 5 ? argv[4] : "single";
    if (mode != "single" && mode != "burst-registered") {
        fprintf(stderr, "unknown mode %s\n", mode.c_str());
        return 1;
    }
    const uint64_t numel = std::strtoull(argv[2], nullptr, 10);
    const uint64_t P = 256, batch_max = 64;
    if (mode == "single" && !std::getenv("PER_LTU_NO_SETUP_CHECK")) {
        // a per-packet worker asks the factory's policy at setup, so a name that
        // refuses per-packet calls fails here, not at its first packet
        int per_ltu = -1;
        try {
            per_ltu = PrePostProcessor::PerLtuCalls(argv[1]);
        } catch (const SwitchMLFatal& e) {
            printf("FAILED %s\n", e.what());
            return 1;
        }
        if (per_ltu < 0) {
            printf("FAILED '%s' is not a valid prepostprocessor.\n", argv[1]);
            return 1;
        }
        if (per_ltu == 0) {
            printf("REFUSED at setup: prepostprocessor '%s' takes the bulk hooks (PreprocessBulk / "
                   "PostprocessBulk) or the burst hooks (PreprocessBurst / PostprocessBurst / "
                   "PostprocessReuseBurst), not one PreprocessSingle / PostprocessSingle per packet; set "
                   "prepostprocessor = hip_exponent_quantizer to accept per-packet launches\n", argv[1]);
            return 3;
        }
    }
    Config cfg;
    cfg.general_.prepostprocessor = argv[1];
    cfg.general_.packet_numel = P;
    cfg.general_.num_workers = 1;
    std::vector<float> host(numel);
    for (uint64_t i = 0; i < numel; i++) host[i] = (float)i * ((i & 1) ? -1.f : 1.f);
    float *d_in = nullptr, *d_out = nullptr;
    int32_t* ring = nullptr;
    uint8_t* extra = nullptr;
    int rc = 0;
    int32_t* reg_ring = nullptr;
    uint8_t* reg_extra = nullptr;
    try {
        ok(hipMalloc(&d_in, numel * 4), "hipMalloc");
        ok(hipMalloc(&d_out, numel * 4), "hipMalloc");
        ok(hipMemcpy(d_in, host.data(), numel * 4, hipMemcpyHostToDevice), "hipMemcpy");
        if (mode == "single") {
            ok(hipHostMalloc(&ring, batch_max * P * 4, hipHostMallocDefault), "hipHostMalloc");
            ok(hipHostMalloc(&extra, batch_max * 2, hipHostMallocDefault), "hipHostMalloc");
        } else {
            reg_ring = static_cast<int32_t*>(std::aligned_alloc(4096, batch_max * P * 4));
            reg_extra = static_cast<uint8_t*>(std::aligned_alloc(4096, 4096));
            if (!reg_ring || !reg_extra) throw SwitchMLFatal("aligned_alloc");
            ok(hipHostRegister(reg_ring, batch_max * P * 4, hipHostRegisterMapped), "hipHostRegister");
            ok(hipHostRegister(reg_extra, 4096, hipHostRegisterMapped), "hipHostRegister");
            ring = reg_ring;
            extra = reg_extra;
            void *dr = nullptr, *dx = nullptr;
            ok(hipHostGetDevicePointer(&dr, reg_ring, 0), "hipHostGetDevicePointer");
            ok(hipHostGetDevicePointer(&dx, reg_extra, 0), "hipHostGetDevicePointer");
            printf("registered ring host %p device %p, extras host %p device %p\n", (void*)reg_ring, dr,
                   (void*)reg_extra, dx);
        }
        auto ppp = PrePostProcessor::CreateInstance(cfg, 0, P * 4, batch_max);
        JobSlice js{nullptr, Tensor{d_in, d_out, numel, FLOAT32}};
        const uint64_t B = ppp->SetupJobSlice(&js);
        const uint64_t b = std::min(B, batch_max);
        const uint64_t total = B + (ppp->NeedsExtraBatch() ? b : 0);
        if (mode == "single") {
            for (uint64_t p = 0; p < b; p++) ppp->PreprocessSingle(p, ring + (p % b) * P, extra + (p % b) * 2);
            for (uint64_t p = 0; p < total; p++) {   // in-order delivery; W = 1: ProcessPacket is the identity
                ppp->PostprocessSingle(p, ring + (p % b) * P, extra + (p % b) * 2);
                if (p + b < total) ppp->PreprocessSingle(p + b, ring + (p % b) * P, extra + (p % b) * 2);
            }
        } else {
            std::vector<uint64_t> ids(b);
            std::vector<void*> ents(b), exs(b);
            for (uint64_t s = 0; s < b; s++) {
                ids[s] = s;
                ents[s] = ring + s * P;
                exs[s] = extra + s * 2;
            }
            ppp->PreprocessBurst((uint32_t)b, ids.data(), ents.data(), exs.data());
            for (uint64_t p0 = 0; p0 < total; p0 += b) {   // one ring pass per burst
                const uint64_t w = std::min(b, total - p0);
                for (uint64_t s = 0; s < w; s++) ids[s] = p0 + s;
                ppp->PostprocessReuseBurst((uint32_t)w, ids.data(), ents.data(), exs.data(), b, total);
            }
        }
        ppp->CleanupJobSlice();
        ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
        ok(hipMemcpy(host.data(), d_out, numel * 4, hipMemcpyDeviceToHost), "hipMemcpy");
        FILE* f = fopen(argv[3], "wb");
        if (!f || fwrite(host.data(), 4, numel, f) != numel) throw SwitchMLFatal("cannot write output");
        fclose(f);
        printf("OK %s: %lu packets through %s calls\n", argv[1], (unsigned long)total,
               mode == "single" ? "per-LTU" : "burst");
    } catch (const SwitchMLFatal& e) {
        const std::string msg = e.what();
        const bool refused = msg.find("PreprocessSingle: ") == 0 || msg.find("PostprocessSingle: ") == 0;
        printf("%s %s\n", refused ? "REFUSED" : "FAILED", msg.c_str());
        rc = refused ? 3 : 1;
    }
    if (reg_ring) {
        (void)hipHostUnregister(reg_ring);
        std::free(reg_ring);
    } else if (ring) {
        (void)hipHostFree(ring);
    }
    if (reg_extra) {
        (void)hipHostUnregister(reg_extra);
        std::free(reg_extra);
    } else if (extra) {
        (void)hipHostFree(extra);
    }
    if (d_in) (void)hipFree(d_in);
    if (d_out) (void)hipFree(d_out);
    return rc;
}
