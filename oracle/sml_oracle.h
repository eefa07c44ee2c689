/*
 * sml_oracle.h — CPU restatement of SwitchML's CpuExponentQuantizerPPP.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (p4app-switchml_amd/,
 * include/) links or calls this.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker / the
 * reported CPU baseline, never as the measured GPU path.
 *
 * Parity status: the reference client_lib cannot be built in this image
 * (common.h:31 includes <glog/logging.h>; glog is absent and stand-ins are
 * not allowed), so this restatement is pinned only by the reference's own
 * known-answer checks (examples/hello_world/main.cc:58-74 and
 * benchmarks/allreduce_benchmark/main.cc:331-399, both 1 % relative) plus
 * hand-derived vectors from reading ppp.cc.  Bit-level parity with the
 * compiled reference is therefore "parity unpinned" (see DESIGN.md §3).
 *
 * All file:line citations are relative to /root/reference/dev_root/client_lib/src/
 * ("ppp.cc" = prepostprocessors/cpu_exponent_quantizer_ppp.cc).
 */
#ifndef SML_ORACLE_H_
#define SML_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ceil(numel*4 / (packet_numel*4)) — ppp.cc:56-57 */
uint64_t orc_num_blocks(uint64_t numel, uint64_t packet_numel);

/* int8 exponent of one block: max |x| over the block (float '>' compare
 * starting from 0, NaN never selected) then ((bits & 0x7f800000) >> 23) - 126
 * truncated to int8 — ppp.cc:129-154. */
int8_t orc_block_exponent(const float* x, uint64_t n);

/* scale = (float)(double(INT32_MAX) / ((float)W * powf(2, e))) — ppp.cc:257-258 */
float orc_scale(uint16_t num_workers, int8_t exponent);
void orc_scale_lut(uint16_t num_workers, float lut[256]); /* lut[(uint8_t)e] */

/* One element of ppp.cc:103: htonl(std::round(x * s)) where the float->uint32
 * conversion is gcc/x86-64's cvttss2si to a 64-bit register truncated to 32
 * bits (out of int64 range / NaN -> 0).  Returns the BIG-ENDIAN word. */
uint32_t orc_quantize_value(float x, float scale);
/* RNE_VCL mode (VCL=1, ppp.cc:88-99: roundi = cvtps2dq, out of range -> 0x80000000).
 * Parity unpinned: VCL is an un-vendored submodule. */
uint32_t orc_quantize_value_rne(float x, float scale);

/* One element of ppp.cc:240-241: (float)(int32)ntohl(be) / s */
float orc_dequantize_value(uint32_t be_word, float scale);

/* ---- plane-level restatement (one job slice) ----------------------------
 * exps[B]                     int8 exponent of each block
 * payload[B*P]                big-endian int32; entries of the last block past
 *                             numel are written as 0 (reference: stale bytes)
 * global_exps == NULL         -> use the local exponents (loopback / W=1 dummy)
 * rounding: 0 = HALF_AWAY (VCL=0 oracle), 1 = RNE_VCL (VCL=1 body, scalar tail)
 */
void orc_exponents(const float* in, uint64_t numel, uint64_t P, int8_t* exps);
void orc_quantize(const float* in, uint64_t numel, uint64_t P, uint16_t num_workers,
                  const int8_t* global_exps, int rounding, uint32_t* payload_be);
void orc_dequantize(const uint32_t* payload_be, const int8_t* global_exps, uint64_t numel,
                    uint64_t P, uint16_t num_workers, float* out);

/* INT32 path: pure byteswap, ppp.cc:158-190 / 262-298 */
void orc_bswap32(const uint32_t* in, uint32_t* out, uint64_t n);

/* DummyBackend::ProcessPacket — dummy_backend.cc:72-84: bswap, *= W (wrap), bswap */
void orc_loopback_aggregate(uint32_t* payload_be, uint64_t n, uint16_t num_workers);

/* Software switch — p4/processor.p4:48-54 (bit<32> wrap add) and
 * p4/exponents.p4:48-54 (signed int<8> max). */
void orc_switch_exps(const int8_t* const* exps, int num_workers, uint64_t B, int8_t* out);
void orc_switch_payload(const uint32_t* const* payload_be, int num_workers, uint64_t n, uint32_t* out);

/* FifoScheduler::GetJobSlice geometry — schedulers/fifo_scheduler.cc:93-109 */
void orc_slice(uint64_t numel, int num_slices, int t, uint64_t* offset, uint64_t* slice_numel);

/* ---- packet-stream driver (DummyWorkerThread order) ----------------------
 * Runs one job through T worker "threads" (sequentially, or on T pthreads when
 * threaded != 0) exactly in DummyWorkerThread call order
 * (backends/dummy/dummy_worker_thread.cc:73-177) with in-order delivery:
 * ring of b = min(max_outstanding_packets/T, B) packets, one extra batch of
 * exponent-only packets, PreprocessSingle/PostprocessSingle per packet and
 * DummyBackend::ProcessPacket (x num_workers) in between.  in == out is allowed.
 * This is the CPU baseline the bench reports.  Returns 0 on success. */
int orc_dummy_allreduce(const float* in, float* out, uint64_t numel, uint64_t P,
                        uint32_t max_outstanding_packets, int num_worker_threads,
                        uint16_t num_workers, int threaded, int mode);
/* mode: ORC_MODE_ROUNDTRIP runs the full packet loop (exponent, quantize+pack,
 * loopback, dequantize); ORC_MODE_PREPROCESS runs only the PreprocessSingle
 * calls of that loop (exponent + quantize+pack into the ring; the scale of
 * block p is stored as the loopback would return it) — the quantize+pack
 * CPU baseline. */
/* Same, with vcl = 1: the reference's VCL=1 build (its default), whose
 * 16-element vector loops are restated with SSE2 intrinsics — the x86-64
 * baseline it is compiled for (client_lib/Makefile:113-120, no -m flags).
 * RNE body / scalar tail, like orc_quantize(rounding = 1). */
int orc_dummy_allreduce_ex(const float* in, float* out, uint64_t numel, uint64_t P,
                           uint32_t max_outstanding_packets, int num_worker_threads,
                           uint16_t num_workers, int threaded, int mode, int vcl);
/* Planes of the VCL=1 build (exponents and BE payload), for the cross-check. */
void orc_quantize_vcl(const float* in, uint64_t numel, uint64_t P, uint16_t num_workers,
                      uint32_t* payload_be, int8_t* exps);
#define ORC_MODE_ROUNDTRIP 0
#define ORC_MODE_PREPROCESS 1

/* Same driver but recording the packet stream of ONE slice (T = 1):
 * pkt_exps[B+b] (byte 0 of the 2-byte extra-info slot at send time) and
 * pkt_payload[(B+b)*P] (BE words at send time; 0 where the reference leaves the
 * ring stale).  Lets tests map planes <-> packet stream. */
int orc_dummy_packet_stream(const float* in, uint64_t numel, uint64_t P,
                            uint32_t batch_max, uint16_t num_workers,
                            int8_t* pkt_exps, uint32_t* pkt_payload, float* out);

/* DPDK frame builder restatement — BuildPacket
 * (backends/dpdk/dpdk_worker_thread_utils.inc:67-135), PktId2PoolIndex (:42-52),
 * DPDK's rte_ipv4_phdr_cksum / rte_raw_cksum (DPDK 20.x, the reference's
 * un-vendored submodule; published algorithm: ones-complement 16-bit sum of
 * the 12-byte pseudo header, folded, not inverted) and PreprocessSingle per
 * packet.  params layout = sml_frame_params of include/switchml_hip.h.
 * Bytes the reference leaves stale are written as 0. */
typedef struct orc_frame_params {
    uint8_t dst_mac[6];
    uint8_t src_mac[6];
    uint32_t src_ip_be, dst_ip_be;
    uint16_t src_port_be, dst_port_be;
    uint64_t job_id;
    uint32_t pool_index_start, pool_index_shift, max_outstanding_pkts;
} orc_frame_params;
uint16_t orc_pkt_id_to_pool_index(uint64_t pkt_id, uint32_t start, uint32_t shift, uint32_t mop);
int orc_build_frames(const float* in, uint64_t numel, uint64_t P, uint16_t num_workers,
                     const int8_t* global_exps, uint32_t batch_max, const orc_frame_params* prm,
                     uint8_t* frames, uint64_t stride);
/* INT32 job slices: B frames (no extra batch), payload = htonl of block p's
 * words (ppp.cc:158-190), and the receive loop with the INT32 PostprocessSingle
 * (ntohl into out, ppp.cc:262-298); `seen` (uint8[B]) carries over. */
int orc_build_frames_i32(const int32_t* in, uint64_t numel, uint64_t P, const orc_frame_params* prm,
                         uint8_t* frames, uint64_t stride);
void orc_unpack_frames_i32(const uint8_t* frames, uint64_t num_frames, uint64_t stride, uint64_t numel,
                           uint64_t P, uint64_t job_id, uint8_t* seen, int32_t* out, uint64_t counts[2]);
/* Receive loop of DpdkWorkerThread + PostprocessSingle over received frames
 * (dpdk_worker_thread.cc:300-345, ppp.cc:197-260).  counts[0] += accepted,
 * counts[1] += discarded; exps (int8[B]) and seen (uint8[B + b], the rx
 * bitmap) in/out across the calls of one slice. */
void orc_dequantize_frames(const uint8_t* frames, uint64_t num_frames, uint64_t stride, uint64_t numel,
                           uint64_t P, uint16_t num_workers, uint32_t batch_max, uint64_t job_id,
                           int8_t* exps, uint8_t* seen, float* out, uint64_t counts[2]);

/* glibc random()/rand() TYPE_3 generator restated (srand(seed) then n calls),
 * and the reference's random-float generator built on it:
 * bits = (r%2)<<31 | (r%254)<<23 | r%(1<<23)  (allreduce_benchmark/main.cc:197-205). */
void orc_glibc_rand(uint32_t seed, uint64_t n, int32_t* out);
void orc_ref_random_floats(uint32_t seed, uint64_t n, float* out);

#ifdef __cplusplus
}
#endif
#endif
