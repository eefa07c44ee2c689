// collnet_bench.cc — configs[4] through the RCCL CollNet plugin table, driven
// from native code the way RCCL's proxy thread drives it (no Python between
// the calls): dlopen librccl-net-switchml.so, resolve ncclCollNetPlugin_v6,
// init / devices / getProperties / listen / connect (one rank), regMr, then
// per iteration post every bucket's iallreduce and poll test() until all are
// done (switchml_plugin.cc:293-387; RCCL keeps several requests in flight).
//
// Buckets: ResNet-50's 25,557,032 fp32 gradients in DDP's 25 MiB buckets
// (3 x 6,553,600 + 5,896,232; not in the reference, parity-unpinned sizes).
// Placements: device buffers (NCCL_PTR_CUDA) and pinned host buffers
// (NCCL_PTR_HOST, what the reference's plugin is handed).  The plugin's
// backend comes from SWITCHML_CONFIG_INI / switchml.cfg; with the loopback
// backend SWITCHML_COLLNET_LOOPBACK=1 must be set (init refuses otherwise).
//
// Output: one JSON line — median ms per iteration and fp32 GB/s per
// placement, and whether both placements produced the same bytes.
//
// Usage: collnet_bench [iterations=20] [plugin path]
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "collnet_abi.h"

namespace {

#define HIP_OK(x)                                                                             \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "collnet_bench: %s: %s\n", #x, hipGetErrorString(e_));            \
            exit(2);                                                                          \
        }                                                                                     \
    } while (0)

#define NCCL_OK(x)                                                                            \
    do {                                                                                      \
        ncclResult_t r_ = (x);                                                                \
        if (r_ != ncclSuccess) {                                                              \
            fprintf(stderr, "collnet_bench: %s returned ncclResult_t %d\n", #x, (int)r_);     \
            exit(3);                                                                          \
        }                                                                                     \
    } while (0)

void quiet_logger(ncclDebugLogLevel, unsigned long, const char*, int, const char*, ...) {}

const int kBuckets[] = {6553600, 6553600, 6553600, 5896232};
constexpr int kNumBuckets = 4;

struct Placement {
    std::vector<float*> send, recv;
    std::vector<void*> mh;
};

// One iteration: every bucket posted, then polled to completion.
void iteration(const ncclCollNet_v6_t* t, void* coll, Placement& p) {
    void* req[kNumBuckets];
    for (int i = 0; i < kNumBuckets; i++)
        NCCL_OK(t->iallreduce(coll, p.send[i], p.recv[i], kBuckets[i], ncclFloat32, ncclSum, p.mh[i], p.mh[i],
                              &req[i]));
    int left = kNumBuckets;
    bool done[kNumBuckets] = {};
    while (left) {
        for (int i = 0; i < kNumBuckets; i++) {
            if (done[i]) continue;
            int d = 0, size = 0;
            NCCL_OK(t->test(req[i], &d, &size));
            if (d) {
                if (size != kBuckets[i] * 4) {
                    fprintf(stderr, "collnet_bench: bucket %d completed with size %d\n", i, size);
                    exit(4);
                }
                done[i] = true;
                left--;
            }
        }
    }
}

double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

}  // namespace

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20;
    const char* path = argc > 2 ? argv[2] : "librccl-net-switchml.so";
    void* so = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!so) {
        fprintf(stderr, "collnet_bench: dlopen %s: %s\n", path, dlerror());
        return 1;
    }
    auto* t = static_cast<const ncclCollNet_v6_t*>(dlsym(so, "ncclCollNetPlugin_v6"));
    if (!t) {
        fprintf(stderr, "collnet_bench: %s exports no ncclCollNetPlugin_v6\n", path);
        return 1;
    }
    NCCL_OK(t->init(quiet_logger));
    int ndev = 0;
    NCCL_OK(t->devices(&ndev));
    ncclNetProperties_v6_t props;
    NCCL_OK(t->getProperties(0, &props));
    char handle[NCCL_NET_HANDLE_MAXSIZE] = {};
    void* lcomm = nullptr;
    NCCL_OK(t->listen(0, handle, &lcomm));
    void* handles[1] = {handle};
    void* coll = nullptr;
    NCCL_OK(t->connect(handles, 1, 0, lcomm, &coll));

    size_t total = 0;
    for (int n : kBuckets) total += (size_t)n;
    // Deterministic gradient-like data (N(0, 1e-3)), the same for both placements.
    std::vector<std::vector<float>> host(kNumBuckets);
    std::mt19937 rng(7);
    std::normal_distribution<float> nd(0.f, 1e-3f);
    for (int i = 0; i < kNumBuckets; i++) {
        host[i].resize(kBuckets[i]);
        for (float& v : host[i]) v = nd(rng);
    }
    Placement dev, pin;
    for (int i = 0; i < kNumBuckets; i++) {
        const size_t bytes = (size_t)kBuckets[i] * 4;
        float *ds, *dr, *hs, *hr;
        HIP_OK(hipMalloc(&ds, bytes));
        HIP_OK(hipMalloc(&dr, bytes));
        HIP_OK(hipHostMalloc(&hs, bytes, hipHostMallocDefault));
        HIP_OK(hipHostMalloc(&hr, bytes, hipHostMallocDefault));
        HIP_OK(hipMemcpy(ds, host[i].data(), bytes, hipMemcpyHostToDevice));
        memcpy(hs, host[i].data(), bytes);
        dev.send.push_back(ds);
        dev.recv.push_back(dr);
        pin.send.push_back(hs);
        pin.recv.push_back(hr);
        void* mh;
        NCCL_OK(t->regMr(coll, ds, (int)bytes, NCCL_PTR_CUDA, &mh));
        dev.mh.push_back(mh);
        NCCL_OK(t->regMr(coll, hs, (int)bytes, NCCL_PTR_HOST, &mh));
        pin.mh.push_back(mh);
    }
    HIP_OK(hipDeviceSynchronize());   // the buffers are ready before they are posted (as under RCCL)

    double ms[2];
    const char* names[2] = {"device", "pinned_host"};
    Placement* pl[2] = {&dev, &pin};
    for (int k = 0; k < 2; k++) {
        for (int w = 0; w < 3; w++) iteration(t, coll, *pl[k]);
        std::vector<double> v;
        for (int it = 0; it < iters; it++) {
            const auto a = std::chrono::steady_clock::now();
            iteration(t, coll, *pl[k]);
            v.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count());
        }
        ms[k] = median(v);
    }
    // both placements ran the same iterations on the same data: same bytes
    bool agree = true;
    for (int i = 0; i < kNumBuckets && agree; i++) {
        std::vector<float> d(kBuckets[i]);
        HIP_OK(hipMemcpy(d.data(), dev.recv[i], (size_t)kBuckets[i] * 4, hipMemcpyDeviceToHost));
        agree = memcmp(d.data(), pin.recv[i], (size_t)kBuckets[i] * 4) == 0;
    }
    printf("{\"what\": \"configs[4] ResNet-50 buckets through ncclCollNetPlugin_v6 from native code (RCCL-proxy "
           "call order)\", \"params\": %zu, \"buckets\": [%d, %d, %d, %d], \"iterations\": %d",
           total, kBuckets[0], kBuckets[1], kBuckets[2], kBuckets[3], iters);
    for (int k = 0; k < 2; k++)
        printf(", \"%s\": {\"ms_per_iteration\": %.4f, \"fp32_GBps\": %.2f}", names[k], ms[k],
               4.0 * (double)total / (ms[k] * 1e-3) / 1e9);
    printf(", \"placements_agree\": %s}\n", agree ? "true" : "false");

    for (int k = 0; k < 2; k++)
        for (void* mh : pl[k]->mh) NCCL_OK(t->deregMr(coll, mh));
    NCCL_OK(t->closeColl(coll));
    NCCL_OK(t->closeListen(lcomm));
    for (int i = 0; i < kNumBuckets; i++) {
        (void)hipFree(dev.send[i]);
        (void)hipFree(dev.recv[i]);
        (void)hipHostFree(pin.send[i]);
        (void)hipHostFree(pin.recv[i]);
    }
    return agree ? 0 : 5;
}
