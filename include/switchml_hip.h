/*
 * switchml_hip.h — C-ABI of the MI355X-native SwitchML end-host
 * pre/post-processor (exponent quantizer) and its loopback/switch helpers.
 *
 * This is the drop-in boundary for the hot path of SwitchML's client_lib:
 * what `CpuExponentQuantizerPPP` (client_lib/src/prepostprocessors/
 * cpu_exponent_quantizer_ppp.{h,cc}) does one 1 KiB LTU at a time on the
 * CPU, these entry points do for a whole job slice at once on the GPU — the
 * "bulk" hooks the reference reserved in prepostprocessor.h:112-116.
 *
 * Conventions
 *  - plain C types only; every pointer argument named d_* is DEVICE memory
 *    (hipMalloc / torch CUDA tensor); `stream` is a hipStream_t passed as
 *    void* (NULL = the legacy default stream).  Calls are asynchronous on
 *    that stream, like every HIP launch.
 *  - no exceptions cross this ABI; every entry point returns sml_status_t.
 *    The reference aborts with LOG(FATAL) on a bad data type / PPP name
 *    (ppp.cc:190,297; prepostprocessor.cc:39); here that is an error code.
 *  - "job slice" = one contiguous run of `numel` elements, exactly what a
 *    worker thread receives from FifoScheduler::GetJobSlice
 *    (schedulers/fifo_scheduler.cc:93-109).  Blocks (LTUs) restart at the
 *    slice start.  Block k covers elements [k*P, min((k+1)*P, numel)).
 *  - planes: the per-packet exponent plane `exps[B]` (int8, byte 0 of the
 *    reference's 2-byte extra-info slot) and the payload plane `payload[B*P]`
 *    (int32, big-endian by default = the packet's wire bytes).  Packet p of
 *    the reference's stream carries exps[p] (p < B) and payload block p-b
 *    (p >= b); see DESIGN.md §2 and SURVEY.md §8 A6.  Payload words of the
 *    last, partial block past `numel` are written as 0 (the reference
 *    leaves stale ring bytes there).
 *  - B = sml_num_blocks(numel, P) = ceil(numel / P)   (ppp.cc:56-57)
 *
 * All file:line citations are relative to /root/reference/dev_root/.
 */
#ifndef SWITCHML_HIP_H_
#define SWITCHML_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SML_ABI_VERSION 2   /* 2: flags on sml_switch_exps / sml_copy_segments, sml_release_to_peers */

typedef enum {
    SML_OK = 0,
    SML_ERR_INVALID_ARG = 1,   /* null pointer with numel > 0, bad W, ... */
    SML_ERR_UNSUPPORTED = 2,   /* packet_numel not in {64,128,256,512,1024}, bad dtype */
    SML_ERR_ALIGNMENT = 3,     /* payload plane not 16-byte aligned */
    SML_ERR_HIP = 4            /* a HIP runtime call or launch failed */
} sml_status_t;

/* client_lib/src/common.h:51-55 */
typedef enum { SML_FLOAT32 = 0, SML_INT32 = 1 } sml_data_type_t;

/* flags for the quantize / dequantize entry points */
#define SML_FLAG_PAYLOAD_LE   0x1u  /* payload plane in host (little-endian) order: the
                                       form RCCL can sum (switch-sim mode); default is
                                       big-endian wire order as htonl() at ppp.cc:103 */
#define SML_FLAG_ROUND_RNE    0x2u  /* VCL=1 semantics (ppp.cc:88-99): round-to-nearest-even
                                       on the 16-aligned body of each block, scalar
                                       half-away tail; out-of-range -> INT32_MIN.
                                       PARITY UNPINNED (VCL is un-vendored). Default is the
                                       VCL=0 scalar path: roundf half-away-from-zero. */
#define SML_FLAG_PEER_PLANES  0x4u  /* the switch entry points (sml_switch_aggregate,
                                       sml_switch_exps, sml_copy_segments): some input
                                       planes were written by OTHER GPUs (peers' HBM mapped
                                       over xGMI).  Every workgroup performs a system-scope
                                       acquire before its first load, so no copy of a peer
                                       line this GPU cached before the peer rewrote it is
                                       read; the peer must have run sml_release_to_peers
                                       after its writes (memory model). */

int sml_abi_version(void);
const char* sml_status_string(sml_status_t s);
/* Last HIP error string seen by this library on the calling thread ("" if none). */
const char* sml_last_error(void);

/* ceil(numel*4 / (packet_numel*4)) — CpuExponentQuantizerPPP::SetupJobSlice, ppp.cc:54-62 */
uint64_t sml_num_blocks(uint64_t numel, uint32_t packet_numel);

/* Host: scale factors for all 256 int8 exponents, lut[(uint8_t)e] =
 *   (float)(double(INT32_MAX) / (num_workers * powf(2, e)))
 * — the scale PostprocessSingle stores from the received global exponent,
 * ppp.cc:254-260.  num_workers >= 1. */
sml_status_t sml_scale_lut(uint16_t num_workers, float lut[256]);

/* Device: the same 256 scales as computed INSIDE the kernels (test hook that
 * proves the device formula equals sml_scale_lut bit for bit). d_lut: float[256]. */
sml_status_t sml_scale_lut_device(uint16_t num_workers, float* d_lut, void* stream);

/* K2 — exponent plane only: d_exps[k] = int8 exponent of block k (max |x|,
 * NaN skipped, ((bits & 0x7f800000) >> 23) - 126) — the exponent half of
 * PreprocessSingle, ppp.cc:115-156.  Used before the exponent exchange in
 * switch-sim mode (the switch's signed int8 max, p4/exponents.p4:48-54). */
sml_status_t sml_exponents(const float* d_in, uint64_t numel, uint32_t packet_numel,
                           int8_t* d_exps, void* stream);

/* K1 / K3 — quantize + pack, the quantize half of PreprocessSingle
 * (ppp.cc:72-113):  payload[k*P+i] = htonl((int32)roundf(x[k*P+i] * scale(W, e_k)))
 *  - d_global_exps == NULL  (K1, fused): e_k is the block's own exponent, as
 *    the dummy/loopback backend returns it unchanged (dummy_backend.cc:72-84);
 *    d_exps_out (nullable) receives the exponent plane.
 *  - d_global_exps != NULL  (K3): e_k = d_global_exps[k], the switch's
 *    aggregated exponent; d_exps_out must be NULL or equal to it (not written).
 *  d_payload: int32[B*P], 16-byte aligned.  d_in may have any 4-byte alignment
 *  (slices start at arbitrary element offsets). */
sml_status_t sml_quantize_pack(const float* d_in, uint64_t numel, uint32_t packet_numel,
                               uint16_t num_workers, const int8_t* d_global_exps,
                               int32_t* d_payload, int8_t* d_exps_out,
                               uint32_t flags, void* stream);

/* K4 — dequantize the aggregated payload, the dequantize half of
 * PostprocessSingle (ppp.cc:197-251):
 *   out[k*P+i] = (float)(int32)ntohl(payload[k*P+i]) / scale(W, exps[k])
 * (int->float RNE, IEEE division).  Only `numel` outputs are written.
 * d_out may have any 4-byte alignment; d_payload 16-byte aligned. */
sml_status_t sml_dequantize(const int32_t* d_payload, const int8_t* d_exps, uint64_t numel,
                            uint32_t packet_numel, uint16_t num_workers, float* d_out,
                            uint32_t flags, void* stream);

/* INT32 jobs — byte-order conversion only (ppp.cc:158-190 pre, 262-298 post).
 * d_out[i] = bswap32(d_in[i]) for i < numel; in == out allowed. */
sml_status_t sml_bswap_i32(const int32_t* d_in, int32_t* d_out, uint64_t numel, void* stream);

/* K5 — the dummy backend's "switch": every BE payload word is multiplied by
 * num_workers with int32 wrap-around, exponents pass through unchanged
 * (DummyBackend::ProcessPacket, client_lib/src/backends/dummy/dummy_backend.cc:72-84).
 * count = B*P words (stale/zero tails included, as the reference does). */
sml_status_t sml_loopback_aggregate(int32_t* d_payload, uint64_t count, uint16_t num_workers,
                                    uint32_t flags, void* stream);

/* Fused loopback round trip for FLOAT32 (dummy backend, one pass over HBM):
 * exponent -> quantize -> x num_workers -> dequantize, writing d_out[numel]
 * and, when d_payload != NULL, the on-wire payload plane as sent (before the
 * loopback multiply) and d_exps_out.  Bit-identical to K1 -> K5 -> K4. */
sml_status_t sml_roundtrip_loopback(const float* d_in, float* d_out, uint64_t numel,
                                    uint32_t packet_numel, uint16_t num_workers,
                                    int32_t* d_payload, int8_t* d_exps_out,
                                    uint32_t flags, void* stream);

/* The fused round trip over a batch of job slices in ONE launch (the
 * client's worker submits every slice of the jobs queued so far together):
 * slice i is exactly sml_roundtrip_loopback(in, out, numel, ...) — its blocks
 * start at its own first element (FIFO slices, fifo_scheduler.cc:93-109) — and
 * no payload / exponent planes are written.  Any 4-byte alignment; slices
 * must not overlap each other (a slice's in == out is fine); numel == 0
 * slices are skipped.  Flags: SML_FLAG_ROUND_RNE (the payload byte order is
 * not observable here). */
#define SML_MAX_BATCH_SLICES 64
typedef struct sml_slice {
    const float* in;
    float* out;
    uint64_t numel;
} sml_slice;
sml_status_t sml_roundtrip_loopback_batch(const sml_slice* slices, uint32_t num_slices, uint32_t packet_numel,
                                          uint16_t num_workers, uint32_t flags, void* stream);

/* ---- The switch's aggregation ---------------------------
 * K6: what the Tofino pipeline does to W workers' packets for one slot, over
 * whole planes, fused with the worker's dequantize:
 *   d_payload_out[i] = htonl(sum_w ntohl(d_payloads[w][i]))  wrapping bit<32>
 *                      (p4/processor.p4:48-54; LE words with
 *                      SML_FLAG_PAYLOAD_LE: no swaps), i < B*P
 *   d_exps_out[k]    = max_w (int8) d_exps[w][k]   (p4/exponents.p4:48-54)
 *   d_out[i]         = (float)(int32)sum_i / scale(W, e_max[i/P]), i < numel
 *                      (PostprocessSingle, ppp.cc:197-251; W = num_workers)
 * d_payloads / d_exps are HOST arrays of num_workers DEVICE pointers: local
 * buffers, or peers' HBM mapped over xGMI (hipIpcOpenMemHandle) — the
 * peer-to-peer switch.  Any of the three outputs may be NULL (not all);
 * d_exps may be NULL when d_exps_out and d_out are.  Payload planes 16-byte
 * aligned (B*P words each); d_payload_out may alias d_payloads[w].
 * num_workers <= SML_MAX_SWITCH_WORKERS. */
#define SML_MAX_SWITCH_WORKERS 16
sml_status_t sml_switch_aggregate(const int32_t* const* d_payloads, const int8_t* const* d_exps,
                                  uint16_t num_workers, uint64_t numel, uint32_t packet_numel,
                                  int32_t* d_payload_out, int8_t* d_exps_out, float* d_out,
                                  uint32_t flags, void* stream);

/* The switch's exponent half alone (p4/exponents.p4:48-54): d_exps_out[k] =
 * max_w (int8) d_exps[w][k], k < num_blocks — W planes of num_blocks bytes
 * (local or mapped peers' planes; HOST array of DEVICE pointers). */
sml_status_t sml_switch_exps(const int8_t* const* d_exps, uint16_t num_workers, uint64_t num_blocks,
                             int8_t* d_exps_out, uint32_t flags, void* stream);

/* Copy num_words 32-bit words (any 4-byte alignment; either side may be a
 * peer's mapped plane or pinned host memory): the all-gather step of the
 * in-node switch backend.  16-B accesses, the streaming kernels' tile shape. */
sml_status_t sml_copy_words(const void* d_src, void* d_dst, uint64_t num_words, void* stream);

/* Up to SML_MAX_SWITCH_WORKERS copies in ONE launch: d_dsts[i][0..n_i) =
 * d_srcs[i][0..n_i), n_i = num_words[i] (HOST arrays of DEVICE pointers, any
 * 4-byte alignment; segments must not overlap).  The in-node switch's
 * multicast: the tiles are dealt round-robin over the segments, so W peers'
 * shards come over their xGMI links at the same time, not one after another. */
sml_status_t sml_copy_segments(const void* const* d_srcs, void* const* d_dsts, const uint64_t* num_words,
                               uint32_t num_segments, uint32_t flags, void* stream);

/* The writer's half of a hand-off to other GPUs: a system-scope release on
 * every XCD of the stream's device (each XCD's L2 writes its dirty lines back
 * to HBM), ordered after the work already on `stream`.  The in-node switch
 * runs it after the kernels that write planes peers will read, before the
 * stream synchronization that precedes the workers' barrier; the readers'
 * kernels then take SML_FLAG_PEER_PLANES (the acquire).  One small launch. */
sml_status_t sml_release_to_peers(void* stream);

/* ---- per-packet calls, a burst per launch ---------------------------------
 * PreprocessSingle / PostprocessSingle (ppp.cc:69-192, 194-299) for up to
 * SML_MAX_BURST packets of one job slice in ONE launch: the DPDK worker's rx
 * burst (PostprocessSingle per received packet, dpdk_worker_thread.cc:300-345)
 * and the tx burst it refills (ReusePacket -> PreprocessSingle of pkt_id + b,
 * dpdk_worker_thread_utils.inc:134,177), or an RDMA worker's completions
 * (rdma_worker_thread.cc:244,356).  entries[i] / extras[i] are packet i's
 * payload words and 2-byte extra-info slot, anywhere the DEVICE can address
 * (HBM, or pinned host memory such as a NIC's buffer pool) — read / written in
 * place.  Packet q of a FLOAT32 slice: preprocess writes block q - b's
 * quantized big-endian words (q >= b; only the block's real words, a partial
 * block's tail stays as it was) and block q's exponent into byte 0 of the
 * extra slot (q < B); postprocess dequantizes block q - b into `out` (q >= b)
 * and keeps the packet's exponent byte as block q's received exponent in
 * recv_exps[q] (q < B).  INT32 slices: byte swaps, packet q = block q.
 * recv_exps: DEVICE array of B int8 owned by the caller for the slice.  Bit-
 * identical to the per-packet calls in the reference's order; packet ids of a
 * burst are distinct and never include both q and q + b (the reference sends
 * q + b only after receiving q).  Flags: SML_FLAG_ROUND_RNE. */
#define SML_MAX_BURST 64
typedef struct {
    const float* in;          /* the job slice (int32 words for INT32) */
    float* out;
    uint64_t numel;
    uint32_t packet_numel;    /* P */
    uint16_t num_workers;     /* W */
    uint16_t data_type;       /* sml_data_type_t */
    uint64_t batch_num_ltus;  /* b (FLOAT32: the extra batch) */
    int8_t* recv_exps;
    uint32_t count;
    uint32_t flags;
    uint64_t pkt_ids[SML_MAX_BURST];
    void* entries[SML_MAX_BURST];
    void* extras[SML_MAX_BURST];
} sml_packet_burst;
sml_status_t sml_preprocess_burst(const sml_packet_burst* burst, void* stream);
sml_status_t sml_postprocess_burst(const sml_packet_burst* burst, void* stream);

/* The receive loop's two calls on one buffer in ONE launch: for every
 * RECEIVED packet q of the burst, PostprocessSingle(q) and then — when packet
 * q + b exists (q + b < B + b for FLOAT32, q + b < B for INT32; b =
 * batch_num_ltus, the packet window, for both types here) —
 * PreprocessSingle(q + b) into the same entries[i] / extras[i]: DpdkWorkerThread's
 * receive loop, PostprocessSingle then ReusePacket (dpdk_worker_thread.cc:
 * 300-345, dpdk_worker_thread_utils.inc:134,177), and DummyWorkerThread's
 * loop trip (dummy_worker_thread.cc:106-163).  Bit-identical to
 * sml_postprocess_burst followed by sml_preprocess_burst of the ids q + b.
 * With SML_FLAG_PROCESS_PACKET the dummy backend's ProcessPacket (all P words
 * x num_workers, wrapping, exponent unchanged; dummy_backend.cc:72-84) is
 * applied to each packet first, and all P words are written back (the words
 * the preprocess does not rewrite keep the processed values). */
#define SML_FLAG_PROCESS_PACKET 0x8u
sml_status_t sml_exchange_burst(const sml_packet_burst* burst, void* stream);

/* A persistent burst server, for packet buffers in HOST memory (a NIC's
 * mbuf pool in pinned memory): there a burst launch costs a launch, PCIe
 * round trips and a host synchronisation, ≈ 20 µs per burst (DESIGN.md §9
 * F1).  The server is one resident workgroup that polls a doorbell in
 * coherent, device-mapped host memory.  sml_burst_server_submit() writes the
 * burst, rings the doorbell and returns once the burst is complete (it spins
 * on the completion word the server publishes with a system-scope release):
 * the same bytes as sml_preprocess_burst (op SML_BURST_PRE),
 * sml_postprocess_burst (SML_BURST_POST) or sml_exchange_burst
 * (SML_BURST_EXCHANGE, SML_FLAG_PROCESS_PACKET honoured), a wave per packet.
 * The server starts with the first submit, leaves its loop after `idle_ms`
 * (0 = 100) without a burst, or on sml_burst_server_stop(), and is restarted
 * by the next submit; destroy stops it and frees it.  While it runs it
 * occupies one CU and a device-wide synchronisation waits for it, so a
 * caller stops it between job slices.
 * packet_numel and SML_FLAG_ROUND_RNE are fixed per server (a burst with
 * other values is refused); one server per calling thread; the current
 * device is the server's. */
typedef struct sml_burst_server sml_burst_server;
#define SML_BURST_PRE 0u
#define SML_BURST_POST 1u
#define SML_BURST_EXCHANGE 2u
sml_status_t sml_burst_server_create(uint32_t packet_numel, uint32_t flags, uint32_t idle_ms,
                                     sml_burst_server** server_out);
sml_status_t sml_burst_server_submit(sml_burst_server* server, uint32_t op, const sml_packet_burst* burst);
/* Leave the loop now and wait for it (the next submit restarts the server);
 * the server's memory and stream are kept for that. */
sml_status_t sml_burst_server_stop(sml_burst_server* server);
sml_status_t sml_burst_server_destroy(sml_burst_server* server);
/* Start the server now (it idles on the doorbell) instead of on the first
 * submit: takes the launch off the first burst's latency.  A relaunch marks
 * every doorbell rung before it as handled, so a burst that failed (a
 * timeout, a workgroup's idle exit mid-burst) is never replayed. */
sml_status_t sml_burst_server_start(sml_burst_server* server);
/* Fault injection for tests: stop the server, then write `burst` and ring the
 * doorbell for it with no server to answer — the state a failed submit
 * leaves (done < doorbell).  Never used on the data path. */
sml_status_t sml_burst_server_inject_unanswered(sml_burst_server* server, uint32_t op,
                                                const sml_packet_burst* burst);

/* Plane sharing for the peer-to-peer switch: export the allocation holding
 * d_ptr as an IPC handle of sml_ipc_handle_bytes() bytes plus d_ptr's byte
 * offset inside it; open a peer's handle in this process (returns the
 * allocation base: add the offset; the mapping reaches the peer GPU's HBM
 * over xGMI, peer access enabled on first use); close it again. */
uint32_t sml_ipc_handle_bytes(void);
sml_status_t sml_ipc_get_handle(const void* d_ptr, void* handle_out, uint64_t* offset_out);
sml_status_t sml_ipc_open_handle(const void* handle, void** d_ptr_out);
sml_status_t sml_ipc_close_handle(void* d_ptr);

/* ---- DPDK/UDP wire frames --------------------------------
 * The DPDK backend builds one Ethernet frame per packet
 * (client_lib/src/backends/dpdk/dpdk_worker_thread_utils.inc:67-135,
 * BuildPacket): Eth(14) + IPv4(20) + UDP(8) + SwitchML header(8:
 * job_type_size, short_job_id, pkt_id (host order), switch_pool_index (BE))
 * + 2-byte extra info (byte 0 = exponent) + packet_numel BE int32 words at
 * offset 52.  Frame p of a job slice (p in [0, B + b), b = min(batch_max, B))
 * carries exps[p] (p < B) and payload block p - b (p >= b), its pool index
 * PktId2PoolIndex(p, start, shift, max_outstanding) (:42-52).
 * Addresses are given in network byte order, as DpdkBackend::E2eAddress. */
typedef struct sml_frame_params {
    uint8_t dst_mac[6];               /* the switch's MAC */
    uint8_t src_mac[6];               /* the worker thread's MAC */
    uint32_t src_ip_be, dst_ip_be;    /* worker, switch (network order) */
    uint16_t src_port_be, dst_port_be;
    uint64_t job_id;                  /* low 8 bits -> short_job_id */
    uint32_t pool_index_start;        /* switch_pool_index_start of the worker thread */
    uint32_t pool_index_shift;        /* switch_pool_index_shift carried across jobs */
    uint32_t max_outstanding_pkts;    /* per worker thread */
} sml_frame_params;

/* Bytes of one frame: 52 + 4 * packet_numel. */
uint64_t sml_frame_bytes(uint32_t packet_numel);

/* Words of the per-slice rx state (d_state) a receive call needs: FLOAT32
 * (sml_dequantize_frames) max(1, B + b) with b = min(batch_max, B); INT32
 * (sml_unpack_frames_int32, int32 != 0) 2B + 6.  B = ceil(numel / P). */
uint64_t sml_rx_state_words(uint64_t numel, uint32_t packet_numel, uint32_t batch_max, int int32);

/* Fused K1 -> frames: quantize + pack one job slice straight into B + b
 * frames at `frame_stride` bytes apart (>= sml_frame_bytes, multiple of 4).
 * `frames` may be device memory or pinned, device-mapped host memory (the
 * NIC's buffers: the kernel then writes them over PCIe).  d_global_exps as
 * for sml_quantize_pack.  Bytes the reference leaves stale (extra-info byte
 * 1, the exponent of frames p >= B, the payload of frames p < b, IPv4
 * identification/TOS/fragment) are written as 0; IPv4 and UDP checksums are
 * left for NIC offload exactly as BuildPacket does (IP 0, UDP = pseudo-header
 * sum, rte_ipv4_phdr_cksum). */
sml_status_t sml_quantize_pack_frames(const float* d_in, uint64_t numel, uint32_t packet_numel,
                                      uint16_t num_workers, const int8_t* d_global_exps,
                                      uint32_t batch_max, const sml_frame_params* params,
                                      void* frames, uint64_t frame_stride, void* stream);

/* Receive side of the DPDK backend (dpdk_worker_thread.cc:300-345): frames
 * the switch returned for one job slice, `num_frames` of them at
 * `frame_stride` bytes apart, in any order (rx bursts gathered into a ring;
 * device or pinned, device-mapped host memory).  A frame is accepted as the
 * worker's receive loop accepts it: short_job_id (byte 43) equal to
 * (uint8_t)job_id and a pkt_id (bytes 44-47, host order) not received
 * before — in an earlier call for the slice, or earlier in `frames` (the
 * first copy wins, :316-330); a pkt_id >= B + b is discarded too.  Every
 * accepted frame is PostprocessSingle'd (ppp.cc:197-260): frame pkt_id < B
 * gives the global exponent of block pkt_id (byte 50, also stored to
 * d_exps[pkt_id]); frame pkt_id >= b gives the aggregated payload of block
 * k = pkt_id - b (BE words at byte 52), dequantized with exponent k into
 * d_out[k*P .. k*P + min(P, numel - k*P)).  As in the reference, the frame
 * carrying exponent k must come in this call or an earlier one for the slice
 * (the switch returns it first).
 *   d_exps:   int8[B], out (the slice's received global exponents)
 *   d_state:  uint64[B + b], 8-B aligned, the rx bitmap (+ received
 *             exponents): zero-filled by the caller before the slice's first
 *             call (rte_bitmap_reset), persists across its calls
 *   d_counts: uint64[2] {accepted, discarded}, added to; nullable, 8-B aligned
 * Two launches on `stream`: claim (thread per frame), then dequantize +
 * retire the winners (wave per 1024 output elements). */
sml_status_t sml_dequantize_frames(const void* frames, uint64_t num_frames, uint64_t frame_stride,
                                   uint64_t numel, uint32_t packet_numel, uint16_t num_workers,
                                   uint32_t batch_max, uint64_t job_id, int8_t* d_exps,
                                   uint64_t* d_state, float* d_out, uint64_t* d_counts,
                                   void* stream);

/* INT32 job slices (DataType::INT32, common.h:51-55) over the same frames.
 * The INT32 pre/post-processor only reorders bytes and needs no extra batch
 * (NeedsExtraBatch is false, ppp.cc:65-67), so a slice has B frames and frame
 * p carries block p: BuildPacket's headers (as sml_quantize_pack_frames,
 * extra-info bytes 0) and htonl of the block's words (ppp.cc:158-190; words
 * past numel in the last frame are 0). */
sml_status_t sml_pack_frames_int32(const int32_t* d_in, uint64_t numel, uint32_t packet_numel,
                                   const sml_frame_params* params, void* frames, uint64_t frame_stride,
                                   void* stream);

/* The receive loop for an INT32 job slice: acceptance as for
 * sml_dequantize_frames (this job, a pkt_id < B not received before, the
 * first copy wins), and PostprocessSingle's INT32 branch (ppp.cc:262-298):
 * ntohl of the accepted frame's words into d_out[pkt_id*P ..
 * pkt_id*P + min(P, numel - pkt_id*P)).  d_state: uint64[2B + 6] (the rx
 * bitmap, the slice's call sequence, the slice's count of copies that
 * claimed ahead of an earlier copy, two alternating slots of a call's
 * conflict count and dirty-list length, then up to B listed pkt_ids),
 * zeroed per slice (sml_rx_reset), persists across calls; d_counts as for
 * sml_dequantize_frames.  One pass in stream order over the frames (an INT32
 * frame needs no other frame) plus a fix-up over a grid of workgroups that
 * rewrites the listed pkt_ids only (all B state words if the list
 * overflowed), on `stream`;
 * num_frames < 2^31 per call, fewer than 2^32 - 1 calls per slice. */
sml_status_t sml_unpack_frames_int32(const void* frames, uint64_t num_frames, uint64_t frame_stride,
                                     uint64_t numel, uint32_t packet_numel, uint64_t job_id,
                                     uint64_t* d_state, int32_t* d_out, uint64_t* d_counts, void* stream);

/* rte_bitmap_reset for one slice (dpdk_worker_thread.cc, per job slice):
 * zero d_state (uint64[B + b]; for INT32 slices uint64[2B + 6]) before the
 * slice's first sml_dequantize_frames / sml_unpack_frames_int32
 * call.  One async memset on `stream`. */
sml_status_t sml_rx_reset(uint64_t* d_state, uint64_t num_words, void* stream);

/* ncclUint8 buckets of the CollNet plugin (switchml_plugin.cc:318-337,
 * 370-378: "SwitchML does not really support uint8"): each byte widened to an
 * int32 for the INT32 all-reduce, and the summed words narrowed back (mod
 * 256).  Device or device-mapped memory; one launch each on `stream`. */
sml_status_t sml_widen_u8_i32(const uint8_t* d_in, int32_t* d_out, uint64_t n, void* stream);
sml_status_t sml_narrow_i32_u8(const int32_t* d_in, uint8_t* d_out, uint64_t n, void* stream);

/* ---- RDMA messages --------------------------------------
 * The RDMA backend's LTU is a message of msg_numel (1024) elements
 * (rdma_worker_thread.cc:86-88): its payload is block m of the planes built
 * with packet_numel = msg_numel.  The exponent travels in the 32-bit
 * immediate: imm = (msg_id & 0xFFFF) | (exponent byte << 16), byte 3 = 0
 * (rdma_worker_thread.cc:341-356; PreprocessSingle writes byte 2).  Message
 * m in [0, B + b) carries exps[m] for m < B; the byte is 0 for m >= B.
 * d_imm: uint32[B + b] (host byte order, as ibv_send_wr.imm_data is filled).
 * d_exps must not be null (SML_ERR_INVALID_ARG): an INT32 slice has its own
 * entry point below. */
sml_status_t sml_rdma_imm(const int8_t* d_exps, uint64_t num_blocks, uint32_t batch_max,
                          uint32_t* d_imm, void* stream);

/* An INT32 slice's immediates: B messages (no extra batch, ppp.cc:65-67),
 * imm = msg_id & 0xFFFF (the INT32 PreprocessSingle leaves byte 2 alone).
 * d_imm: uint32[B]. */
sml_status_t sml_rdma_imm_int32(uint64_t num_blocks, uint32_t* d_imm, void* stream);

/* Measurement probe (not part of the PPP): copy `bytes` (a multiple of 4 KiB,
 * 16-B aligned buffers) with the quantize kernel's tile shape (K1's slices
 * per wave tile) and access policy (non-temporal loads; non-temporal stores from the payload
 * non-temporal threshold on, default-policy stores below it — the store
 * policy sml_quantize_pack uses for an output plane of `bytes`) — the
 * practical HBM ceiling bench.py reports. */
sml_status_t sml_stream_copy(const void* d_in, void* d_out, uint64_t bytes, void* stream);

/* Fault injection for tests (not part of the PPP): one small kernel that
 * keeps `stream` busy for `microseconds` of the device's wall clock (at most
 * 60 s; SML_ERR_INVALID_ARG above) and then ends on its own — a device that
 * does not finish within a caller's timeout (backend.dummy.stall_worker_thread
 * uses it to exercise the in-node switch's bounded waits), never a hang. */
sml_status_t sml_debug_stall(uint32_t microseconds, void* stream);

/* Launch-geometry knob for experiments: workgroups per launch for the
 * streaming kernels (0 = one 256-thread workgroup per 4 tiles of 1024
 * elements, i.e. no grid-stride).  Process-wide; returns the previous value. */
uint32_t sml_set_grid_limit(uint32_t max_workgroups);

/* Launch-order knob: the streaming kernels permute workgroups so that each
 * of the 8 XCDs sweeps runs of `chunk` consecutive workgroups' data (default
 * 64; 0 = plain blockIdx order).  Process-wide; returns the previous value. */
uint32_t sml_set_xcd_chunk(uint32_t chunk);

/* Tuning knob: slices of 256 elements per wave tile in sml_exponents /
 * sml_quantize_pack (K1/K2/K3): 4, 2 or 1 for every kernel — never below
 * P / 256 — or 0 (the default; any other value restores it): 2, measured
 * fastest for all three on the final kernels.
 * Results are identical for every size.  Returns the
 * previous value. */
uint32_t sml_set_quantize_tile_slices(uint32_t slices);

/* Tuning knob: slices of 256 elements per wave tile in sml_dequantize (K4)
 * and sml_roundtrip_loopback (the fused round trip; P = 1024 keeps 4): 4 or
 * 2 for both, or 0 = the default, 2 for both (as measured).
 * Results are identical for every size.  Returns
 * the previous value. */
uint32_t sml_set_stream_tile_slices(uint32_t slices);

/* Tuning knob: output planes of at least `bytes` bytes are written with
 * non-temporal stores — the payload plane of sml_quantize_pack (K1/K3), the
 * fp32 output of sml_dequantize (K4), sml_roundtrip_loopback and
 * sml_roundtrip_loopback_batch (by the batch's total output), the fp32
 * output of sml_dequantize_frames, the payloads of a device-memory frame set
 * of sml_quantize_pack_frames (host frame sets keep default stores) and the
 * sml_stream_copy probe; default 64 MiB, a quarter of the 256 MiB Infinity
 * Cache — DESIGN.md §4); UINT64_MAX = never, 0 = always.
 * Results are identical either way.  Returns the previous value. */
uint64_t sml_set_payload_nt_threshold(uint64_t bytes);

#ifdef __cplusplus
}
#endif

#endif /* SWITCHML_HIP_H_ */
