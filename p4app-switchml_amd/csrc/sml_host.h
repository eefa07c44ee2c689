// sml_host.h — host-side helpers shared by the C-ABI translation units
// (argument checks, HIP error capture, launch geometry).
#ifndef SML_HOST_H_
#define SML_HOST_H_

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <string.h>

#include <atomic>

#include "sml_device.h"
#include "switchml_hip.h"

namespace sml {

// Process-wide launch knobs and the thread's last HIP error message
// (defined in sml_quantizer.hip).
extern thread_local char g_last_error[256];
extern std::atomic<uint32_t> g_grid_limit;
extern std::atomic<uint32_t> g_xcd_chunk;
extern std::atomic<uint64_t> g_nt_threshold;   // output planes from this size on: non-temporal stores

inline sml_status_t hip_check(hipError_t err) {
    if (err == hipSuccess) return SML_OK;
    strncpy(g_last_error, hipGetErrorString(err), sizeof(g_last_error) - 1);
    return SML_ERR_HIP;
}

inline sml_status_t launch_check() { return hip_check(hipGetLastError()); }

inline bool valid_packet(uint32_t P) {
    return P == 64 || P == 128 || P == 256 || P == 512 || P == 1024;
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }
inline bool aligned4(const void* p) { return ((uintptr_t)p & 3u) == 0; }

inline uint32_t grid_for_tiles(uint64_t ntiles) {
    uint64_t g = (ntiles + kWavesPerBlock - 1) / kWavesPerBlock;
    if (g == 0) g = 1;
    const uint32_t lim = g_grid_limit.load(std::memory_order_relaxed);
    if (lim && g > lim) g = lim;
    if (g > 0x7fffffffull) g = 0x7fffffffull;
    return (uint32_t)g;
}

inline uint32_t grid_for_vec(uint64_t nvec) {
    uint64_t g = (nvec + kBlockThreads - 1) / kBlockThreads;
    const uint32_t lim = g_grid_limit.load(std::memory_order_relaxed);
    uint64_t cap = lim ? lim : 8192;
    if (g > cap) g = cap;
    if (g == 0) g = 1;
    return (uint32_t)g;
}

}  // namespace sml

#endif  // SML_HOST_H_
