// config.h — the configuration keys of the SwitchML client that the
// pre/post-processor path reads (client_lib/src/config.h:35-113 for the
// general section; backend.dummy keys from configs/dummy.cfg), plus this
// build's backend.hip section.  The reference parses INI with
// boost::program_options; here a small INI reader accepts the same files
// (unknown keys such as backend.dpdk.* are ignored with a warning).
#ifndef SWITCHML_AMD_CONFIG_H_
#define SWITCHML_AMD_CONFIG_H_

#include <cstdint>
#include <string>

namespace switchml {

struct GeneralConfig {
    uint16_t rank = 0;
    uint16_t num_workers = 1;
    uint16_t num_worker_threads = 4;
    uint32_t max_outstanding_packets = 256;
    uint64_t packet_numel = 1024;          // code default (config.cc:51); general.cfg ships 256
    std::string backend = "dummy";
    std::string scheduler = "fifo";
    std::string prepostprocessor = "cpu_exponent_quantizer";
    bool instant_job_completion = false;
    std::string controller_ip_str = "127.0.0.1";
    uint16_t controller_port = 50099;
};

struct DummyBackendConfig {
    float bandwidth = 1000.0f;             // Mbps; <= 0 disables the simulated wire time
    bool process_packets = true;           // multiply payloads by num_workers (the "switch")
    // Fault injection for tests (the client-side analogue of the reference's
    // P4 drop simulator, controller/drop_simulator.py): the worker thread with
    // this id fails every slice it is handed without touching the buffers.
    int fail_worker_thread = -1;
    // Fault injection for tests: before each slice it is handed, the worker
    // thread with id stall_worker_thread queues a kernel that keeps its stream
    // busy for stall_ms (sml_debug_stall; at most 60000) — a device that does
    // not finish within backend.xgmi.timeout_ms, which ends on its own.
    int stall_worker_thread = -1;
    uint32_t stall_ms = 0;
};

// MI355X-specific knobs of the loopback backend.
struct HipBackendConfig {
    int device = -1;                       // -1: the caller's current HIP device
    // How a worker thread runs a FLOAT32 job slice:
    //  "bulk"   : K1 quantize+pack -> K5 x num_workers -> K4 dequantize (planes in HBM)
    //  "fused"  : one round-trip kernel, no planes (fastest)
    //  "packet" : the reference's per-LTU PreprocessSingle/PostprocessSingle loop
    //             (DummyWorkerThread order) — API-parity mode, slow by design
    std::string mode = "bulk";
    // Where "packet" mode's ring of b packet buffers lives: "device" (HBM),
    // "pinned" (page-locked host memory, a NIC's DMA buffers) or "pageable"
    // (plain malloc) — the per-LTU calls handle all three (staged or direct).
    std::string packet_ring = "device";
    // Burst calls whose packet buffers are in host memory (pinned ring, a
    // NIC's mbuf pool) go to a persistent burst server (sml_burst_server_*:
    // one resident workgroup polling a doorbell) instead of one launch and a
    // host synchronisation per burst; the server runs for the job slice.
    bool burst_server = false;
    // mode = fused, loopback switch, no simulated wire: ONE worker thread
    // takes every slice of up to batch_jobs queued jobs (at most
    // SML_MAX_BATCH_SLICES slices) and runs them in one kernel launch
    // (sml_roundtrip_loopback_batch) — same FIFO slice geometry and results,
    // one launch instead of num_worker_threads per job.  0: every worker
    // thread launches its own slice (the reference's threading).
    uint32_t batch_jobs = 16;
    // Batched dispatch with a zero-copy (pinned host) job in the round: jobs
    // that arrive within coalesce_us of the previous one join the same
    // launch (PCIe moves more bytes per second in larger launches); 0 = off.
    uint32_t coalesce_us = 20;
    // The quantizer's rounding, as the reference's two client_lib builds do
    // it (client_lib/Makefile:26,113-120): false = the VCL=0 build (roundf,
    // half away from zero, every element; ppp.cc:100-109), true = the VCL=1
    // build (round-to-nearest-even on each packet's 16-element vector body,
    // roundf on its tail, ppp.cc:88-99; SML_FLAG_ROUND_RNE).  A caller who
    // ran the reference's default build sets vcl = true for its bits.
    bool vcl = false;
};

// The in-node switch (general.backend = "xgmi", xgmi_switch.h): W worker
// processes of one node (general.rank, general.num_workers) exchange through
// each other's HBM; `session` names their shared rendezvous segment.
struct XgmiBackendConfig {
    std::string session;
    uint64_t max_slice_numel = 16ull << 20;   // exchange chunk (elements) and plane size per worker thread
    uint64_t timeout_ms = 60000;              // a worker missing a barrier this long fails the slice
    // FLOAT32 exchange direction: false = every worker's K6 READS its shard
    // of the W payload planes over xGMI (pull); true = every worker's K3
    // WRITES each shard of its payload straight into the owner's inbox over
    // xGMI and K6 reads only local HBM (push).  Same bytes; all workers of a
    // session must agree.  The multicast (gather) pulls in both.
    bool push = false;
    // Fault injection for tests: this worker fails right after joining the
    // session (handles published, the workers' barrier passed), as one that
    // cannot map a peer's plane on its first contact with another GPU does.
    bool fail_setup = false;
};

struct BackendConfig {
    DummyBackendConfig dummy;
    HipBackendConfig hip;
    XgmiBackendConfig xgmi;
};

class Config {
  public:
    GeneralConfig general_;
    BackendConfig backend_;

    // Same search order as the reference (config.cc:103-144) when path is
    // empty: /etc/switchml.cfg, ./switchml.cfg, ./switchml-<hostname>.cfg.
    bool LoadFromFile(std::string path = "");
    bool LoadFromString(const std::string& ini);
    // config.cc:154-213 (general part): mop must give every worker thread a
    // packet; mop is rounded to a multiple of num_worker_threads.
    void Validate();
    std::string ToString() const;
    void PrintConfig() const;
};

}  // namespace switchml

#endif  // SWITCHML_AMD_CONFIG_H_
