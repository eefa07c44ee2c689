/*
 * switchml_client.h — C-ABI of the SwitchML client Context (MI355X build).
 *
 * The reference exposes its client only as C++ (client_lib/src/context.h:76-155:
 * switchml::Context::GetInstance / Start / Stop / AllReduceAsync / AllReduce /
 * WaitForAllJobs, and Job::WaitToComplete / GetJobStatus).  This header is
 * the same surface as plain C so any FFI (ctypes, cgo, JNI, N-API) can bind
 * it; C++ callers can use p4app-switchml_amd/csrc/client/context.h directly.
 *
 * Tensors passed to sml_allreduce* may be host or device (HIP) memory.
 * Errors are returned, never thrown: SML_CTX_OK or a negative code; the text
 * of the last failure is available from sml_context_last_error().
 */
#ifndef SWITCHML_CLIENT_H_
#define SWITCHML_CLIENT_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SML_CTX_OK 0
#define SML_CTX_ERR_STATE (-1)    /* wrong context state for the call */
#define SML_CTX_ERR_CONFIG (-2)   /* invalid / missing configuration */
#define SML_CTX_ERR_ARG (-3)
#define SML_CTX_ERR_FAILED (-4)   /* the job FAILED */

/* Context states (context.h ContextState) and job states (job.h JobStatus). */
enum { SML_CTX_CREATED = 0, SML_CTX_STARTING, SML_CTX_RUNNING, SML_CTX_STOPPING, SML_CTX_STOPPED };
enum { SML_JOB_INIT = 0, SML_JOB_QUEUED, SML_JOB_RUNNING, SML_JOB_FINISHED, SML_JOB_FAILED };
/* DataType (common.h:51-55) and AllReduceOperation (job.h:44-46) */
enum { SML_DT_FLOAT32 = 0, SML_DT_INT32 = 1 };
enum { SML_OP_SUM = 0 };

typedef struct sml_job_s* sml_job_t;

/* Start the context.  config_ini: the text of a switchml.cfg (INI with the
 * reference's keys: [general] num_workers, num_worker_threads,
 * max_outstanding_packets, packet_numel, prepostprocessor, ...;
 * [backend.dummy] bandwidth, process_packets; [backend.hip] device, mode).
 * NULL: load switchml.cfg from the reference's search path. */
int sml_context_start(const char* config_ini);
int sml_context_stop(void);
int sml_context_state(void);
const char* sml_context_last_error(void);
/* The effective (validated) configuration as INI text; valid until the next call. */
const char* sml_context_config(void);

/* Context::AllReduceAsync / AllReduce / WaitForAllJobs */
int sml_allreduce_async(void* in_ptr, void* out_ptr, uint64_t numel, int data_type, int op, sml_job_t* job);
int sml_allreduce(void* in_ptr, void* out_ptr, uint64_t numel, int data_type, int op);
int sml_wait_for_all_jobs(void);

/* Job::WaitToComplete / GetJobStatus; every job handle must be released. */
int sml_job_wait(sml_job_t job);   /* SML_CTX_OK if FINISHED, SML_CTX_ERR_FAILED if FAILED */
int sml_job_status(sml_job_t job);
uint64_t sml_job_id(sml_job_t job);
void sml_job_release(sml_job_t job);

/* Stats: out[0] jobs submitted, [1] jobs finished, [2] numel submitted,
 * [3] job slices processed, [4] packets (LTUs) processed incl. extra batch. */
int sml_context_stats(uint64_t out[5]);

/* Whether the PrePostProcessor a factory key names (config key
 * general.prepostprocessor; PrePostProcessor::CreateInstance,
 * client_lib/src/prepostprocessor.cc:32-41) accepts per-LTU calls
 * (PreprocessSingle / PostprocessSingle once per packet): 1 yes
 * ("hip_exponent_quantizer", "bypass"), 0 no — "cpu_exponent_quantizer", the
 * reference's name, maps to the MI355X quantizer driven by its bulk / burst
 * hooks, and its per-LTU calls throw rather than run one launch and host sync
 * per 1 KiB packet — or SML_CTX_ERR_CONFIG for a name the factory rejects.
 * A packet-driven backend (a DPDK / RDMA worker) checks this at setup. */
int sml_ppp_per_ltu_calls(const char* name);

#ifdef __cplusplus
}
#endif

#endif /* SWITCHML_CLIENT_H_ */
