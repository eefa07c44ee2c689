// pcie_probe.hip — host<->device copy ceilings on the GPU box (tools only):
// H2D alone, D2H alone, and both at once on two streams (SDMA engines), with
// pinned host memory, so the host-inclusive pipeline in DESIGN.md §7 can be
// read against what PCIe itself gives.  Prints JSON.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char** argv) {
    const size_t bytes = (size_t)(argc > 1 ? atoi(argv[1]) : 256) << 20;
    const size_t chunk = (size_t)(argc > 2 ? atoi(argv[2]) : 32) << 20;
    void *h_in, *h_out, *d_in, *d_out;
    CK(hipHostMalloc(&h_in, bytes, hipHostMallocDefault));
    CK(hipHostMalloc(&h_out, bytes, hipHostMallocDefault));
    CK(hipMalloc(&d_in, bytes));
    CK(hipMalloc(&d_out, bytes));
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    auto timeit = [&](auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        const int reps = 5;
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; i++) fn();
        CK(hipDeviceSynchronize());
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
    };
    auto h2d = [&] { for (size_t o = 0; o < bytes; o += chunk)
        CK(hipMemcpyAsync((char*)d_in + o, (char*)h_in + o, chunk, hipMemcpyHostToDevice, a)); };
    auto d2h = [&] { for (size_t o = 0; o < bytes; o += chunk)
        CK(hipMemcpyAsync((char*)h_out + o, (char*)d_out + o, chunk, hipMemcpyDeviceToHost, b)); };
    auto both = [&] { h2d(); d2h(); };
    const double t1 = timeit(h2d), t2 = timeit(d2h), t3 = timeit(both);
    printf("{\"bytes\": %zu, \"chunk\": %zu, \"h2d_GBps\": %.2f, \"d2h_GBps\": %.2f, "
           "\"bidir_each_way_GBps\": %.2f}\n", bytes, chunk, bytes / t1 / 1e9, bytes / t2 / 1e9, bytes / t3 / 1e9);
    return 0;
}
