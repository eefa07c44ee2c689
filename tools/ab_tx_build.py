#!/usr/bin/env python3
"""Build frames-tx (k_quantize_frames) variants of the kernel library into
tools/ab/ (sources copied and patched there; tools/ab/ is git-ignored):
  tx_base   the product source
  tx_bf     payload stores of a full tile in a branch-free loop, the four
            slices' scales read from the LDS table before any store
  tx_nohdr  DIAGNOSTIC ONLY (frames wrong): no lane-parallel header stores —
            what do the headers cost?
  fr_w8     k_quantize_frames and k_rx_apply held to 8 waves per SIMD
            (amdgpu_waves_per_eu): both are SGPR-limited to 7 otherwise
  tx_w8     the same for k_quantize_frames only
  sw_w8     the same for K6 k_switch_aggregate (6-7 waves otherwise)
  rx_vec    rx apply reads its state words with vector (broadcast) loads
  rx_vec_w8 rx_vec held to 8 waves per SIMD
  k1_ntstore K1's payload stores non-temporal (tools/ab_store_size.py)
  rx_ntout  rx apply's fp32 output stores non-temporal
Timed by tools/ab_frames.py on the GPU (AB_NOCHECK=1 when tx_nohdr is in)."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "p4app-switchml_amd")
AB = os.path.join(ROOT, "tools", "ab")

PAYLOAD = """        // payloads
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4;
            if (idx >= padded) continue;"""
PAYLOAD_BF = """        // payloads
        if (base + kTileElems <= padded) {
            float s[kU];
#pragma unroll
            for (int u = 0; u < kU; u++) {
                int e = eloc[u];
                if constexpr (GLOBAL) e = a.gexp[(base + (uint64_t)(u * kWave + lane) * 4) / P];
                s[u] = lut[(uint8_t)e];
            }
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4;
                const uint64_t k = idx / P;
                const u4 q = quantize4<false>(v[u], s[u], idx, 0);
                uint32_t* dst = reinterpret_cast<uint32_t*>(a.frames + (k + a.b) * a.stride + 52) + (idx - k * P);
                *reinterpret_cast<u4a*>(dst) = u4a{bswap(q.x), bswap(q.y), bswap(q.z), bswap(q.w)};
            }
            continue;
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const uint64_t idx = base + (uint64_t)(u * kWave + lane) * 4;
            if (idx >= padded) continue;"""
HDR = """            if (lane < 48) {
                if (j < kPk && pk0 + j < a.nblocks) {"""
NOHDR = """            if (lane < 48) {
                if (j < kPk && pk0 + j < a.nblocks && a.W == 0xffffu) {"""


def build(name, patches=()):
    d = os.path.join(AB, name)
    if os.path.isdir(d):
        shutil.rmtree(d)
    shutil.copytree(os.path.join(PKG, "csrc"), os.path.join(d, "csrc"))
    for patch in patches:
        fname, old, new = patch if len(patch) == 3 else ("sml_frames.hip",) + tuple(patch)
        f = os.path.join(d, "csrc", fname)
        s = open(f).read()
        assert s.count(old) == 1, old
        open(f, "w").write(s.replace(old, new))
    objs = []
    for k in ("sml_quantizer", "sml_frames", "sml_switch"):
        o = os.path.join(d, k + ".o")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                        "-I" + os.path.join(ROOT, "include"), "-fno-gpu-rdc", "-c", "-o", o,
                        os.path.join(d, "csrc", k + ".hip")], check=True)
        objs.append(o)
    out = os.path.join(AB, name + ".so")
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-fno-gpu-rdc", "-o", out] + objs,
                   check=True)
    shutil.rmtree(d)
    print(out)


TXK = "__global__ __launch_bounds__(kBlockThreads) void k_quantize_frames(FrameArgs a) {"
RXK = "__global__ __launch_bounds__(kBlockThreads) void k_rx_apply(RxArgs a) {"
W8 = "__attribute__((amdgpu_waves_per_eu(8, 8))) "
RXO = "            if (a.numel - off >= 4 && ((uintptr_t)p & 15u) == 0) *reinterpret_cast<f4*>(p) = o[u];"
RXS = "        if constexpr (kChunksPerFrame >= kWave) {"
SWK = "__global__ __launch_bounds__(kBlockThreads) void k_switch_aggregate(SwitchArgs a) {"

VARIANTS = {"tx_base": (), "tx_bf": ((PAYLOAD, PAYLOAD_BF),), "tx_nohdr": ((HDR, NOHDR),),
            # occupancy: both frames kernels are SGPR-limited to 7 waves per SIMD (106 SGPRs)
            "fr_w8": ((TXK, TXK.replace("__global__ ", "__global__ " + W8)),
                      (RXK, RXK.replace("__global__ ", "__global__ " + W8))),
            "tx_w8": ((TXK, TXK.replace("__global__ ", "__global__ " + W8)),),
            # rx apply: non-temporal fp32 output stores
            "rx_ntout": ((RXO, RXO.replace("*reinterpret_cast<f4*>(p) = o[u];",
                                            "__builtin_nontemporal_store(o[u], reinterpret_cast<f4*>(p));")),),
            # K1: non-temporal payload stores (sml_device.h store_payload)
            "k1_ntstore": (("sml_device.h", "__device__ __forceinline__ void store_payload(u4* dst, u4 q) { *dst = q; }",
                            "__device__ __forceinline__ void store_payload(u4* dst, u4 q) { __builtin_nontemporal_store(q, dst); }"),),
            # rx apply: state words by (broadcast) vector loads instead of scalar loads, so the
            # SGPR budget fits 8 waves without spilling into the loop; with and without the hint
            "rx_vec": ((RXS, RXS.replace("kChunksPerFrame >= kWave", "false && kChunksPerFrame >= kWave")),),
            "rx_vec_w8": ((RXS, RXS.replace("kChunksPerFrame >= kWave", "false && kChunksPerFrame >= kWave")),
                          (RXK, RXK.replace("__global__ ", "__global__ " + W8))),
            # K6 (switch aggregate): 6-7 waves per SIMD by its SGPRs / VGPRs
            "sw_w8": (("sml_switch.hip", SWK, SWK.replace("__global__ ", "__global__ " + W8)),)}

if __name__ == "__main__":
    os.makedirs(AB, exist_ok=True)
    for name in sys.argv[1:] or list(VARIANTS):
        build(name, VARIANTS[name])
