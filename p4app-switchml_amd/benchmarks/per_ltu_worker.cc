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
// Usage: per_ltu_worker <prepostprocessor> <numel> <out.f32>
//   input x[i] = float(i) * (-1)^i (allreduce_benchmark/main.cc:207-212) in HBM;
//   the dequantized output is written to <out.f32>.
// Exit 0: done; 3: the PPP refused per-packet calls (message on stdout);
// 1: any other failure.
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
    if (argc != 4) {
        fprintf(stderr, "usage: %s <prepostprocessor> <numel> <out.f32>\n", argv[0]);
        return 1;
    }
    const uint64_t numel = std::strtoull(argv[2], nullptr, 10);
    const uint64_t P = 256, batch_max = 64;
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
    try {
        ok(hipMalloc(&d_in, numel * 4), "hipMalloc");
        ok(hipMalloc(&d_out, numel * 4), "hipMalloc");
        ok(hipMemcpy(d_in, host.data(), numel * 4, hipMemcpyHostToDevice), "hipMemcpy");
        ok(hipHostMalloc(&ring, batch_max * P * 4, hipHostMallocDefault), "hipHostMalloc");
        ok(hipHostMalloc(&extra, batch_max * 2, hipHostMallocDefault), "hipHostMalloc");
        auto ppp = PrePostProcessor::CreateInstance(cfg, 0, P * 4, batch_max);
        JobSlice js{nullptr, Tensor{d_in, d_out, numel, FLOAT32}};
        const uint64_t B = ppp->SetupJobSlice(&js);
        const uint64_t b = std::min(B, batch_max);
        const uint64_t total = B + (ppp->NeedsExtraBatch() ? b : 0);
        for (uint64_t p = 0; p < b; p++) ppp->PreprocessSingle(p, ring + (p % b) * P, extra + (p % b) * 2);
        for (uint64_t p = 0; p < total; p++) {   // in-order delivery; W = 1: ProcessPacket is the identity
            ppp->PostprocessSingle(p, ring + (p % b) * P, extra + (p % b) * 2);
            if (p + b < total) ppp->PreprocessSingle(p + b, ring + (p % b) * P, extra + (p % b) * 2);
        }
        ppp->CleanupJobSlice();
        ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
        ok(hipMemcpy(host.data(), d_out, numel * 4, hipMemcpyDeviceToHost), "hipMemcpy");
        FILE* f = fopen(argv[3], "wb");
        if (!f || fwrite(host.data(), 4, numel, f) != numel) throw SwitchMLFatal("cannot write output");
        fclose(f);
        printf("OK %s: %lu packets through per-LTU calls\n", argv[1], (unsigned long)total);
    } catch (const SwitchMLFatal& e) {
        const std::string msg = e.what();
        const bool refused = msg.find("PreprocessSingle: ") == 0 || msg.find("PostprocessSingle: ") == 0;
        printf("%s %s\n", refused ? "REFUSED" : "FAILED", msg.c_str());
        rc = refused ? 3 : 1;
    }
    if (ring) (void)hipHostFree(ring);
    if (extra) (void)hipHostFree(extra);
    if (d_in) (void)hipFree(d_in);
    if (d_out) (void)hipFree(d_out);
    return rc;
}
