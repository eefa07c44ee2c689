// capi_context.cc — include/switchml_client.h over switchml::Context.
#include <memory>
#include <string>

#include "context.h"
#include "prepostprocessor.h"
#include "switchml_client.h"

using namespace switchml;

struct sml_job_s {
    std::shared_ptr<Job> job;
};

namespace {
thread_local std::string g_err;
thread_local std::string g_cfg;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
}  // namespace

extern "C" {

const char* sml_context_last_error(void) { return g_err.c_str(); }

int sml_context_start(const char* config_ini) {
    try {
        Context& ctx = Context::GetInstance();
        bool ok;
        if (config_ini) {
            Config cfg;
            cfg.LoadFromString(config_ini);
            ok = ctx.Start(&cfg);
        } else {
            ok = ctx.Start(nullptr);
        }
        return ok ? SML_CTX_OK : fail(SML_CTX_ERR_STATE, "context is not in the CREATED/STOPPED state");
    } catch (const std::exception& e) {
        return fail(SML_CTX_ERR_CONFIG, e.what());
    }
}

int sml_context_stop(void) {
    try {
        Context::GetInstance().Stop();
        return SML_CTX_OK;
    } catch (const std::exception& e) {
        return fail(SML_CTX_ERR_STATE, e.what());
    }
}

int sml_context_state(void) { return (int)Context::GetInstance().GetContextState(); }

const char* sml_context_config(void) {
    g_cfg = Context::GetInstance().GetConfig().ToString();
    return g_cfg.c_str();
}

int sml_allreduce_async(void* in_ptr, void* out_ptr, uint64_t numel, int data_type, int op, sml_job_t* job) {
    if (!job || (data_type != SML_DT_FLOAT32 && data_type != SML_DT_INT32) || op != SML_OP_SUM)
        return fail(SML_CTX_ERR_ARG, "invalid argument");
    if (numel && (!in_ptr || !out_ptr)) return fail(SML_CTX_ERR_ARG, "null tensor pointer");
    try {
        auto j = Context::GetInstance().AllReduceAsync(in_ptr, out_ptr, numel, (DataType)data_type, SUM);
        *job = new sml_job_s{j};
        return SML_CTX_OK;
    } catch (const std::exception& e) {
        return fail(SML_CTX_ERR_STATE, e.what());
    }
}

int sml_allreduce(void* in_ptr, void* out_ptr, uint64_t numel, int data_type, int op) {
    sml_job_t j = nullptr;
    int rc = sml_allreduce_async(in_ptr, out_ptr, numel, data_type, op, &j);
    if (rc != SML_CTX_OK) return rc;
    rc = sml_job_wait(j);
    sml_job_release(j);
    return rc;
}

int sml_wait_for_all_jobs(void) {
    try {
        Context::GetInstance().WaitForAllJobs();
        return SML_CTX_OK;
    } catch (const std::exception& e) {
        return fail(SML_CTX_ERR_STATE, e.what());
    }
}

int sml_job_wait(sml_job_t job) {
    if (!job) return fail(SML_CTX_ERR_ARG, "null job");
    job->job->WaitToComplete();
    return job->job->GetJobStatus() == FINISHED ? SML_CTX_OK : fail(SML_CTX_ERR_FAILED, "job failed");
}

int sml_job_status(sml_job_t job) { return job ? (int)job->job->GetJobStatus() : SML_CTX_ERR_ARG; }

uint64_t sml_job_id(sml_job_t job) { return job ? job->job->id_ : ~0ull; }

void sml_job_release(sml_job_t job) { delete job; }

int sml_context_stats(uint64_t out[5]) {
    if (!out) return SML_CTX_ERR_ARG;
    Stats& s = Context::GetInstance().GetStats();
    out[0] = s.jobs_submitted();
    out[1] = s.jobs_finished();
    out[2] = s.numel_submitted();
    out[3] = s.slices_processed();
    out[4] = s.ltus_processed();
    return SML_CTX_OK;
}

int sml_ppp_per_ltu_calls(const char* name) {
    if (!name) return SML_CTX_ERR_ARG;
    const int r = PrePostProcessor::PerLtuCalls(name);
    return r < 0 ? fail(SML_CTX_ERR_CONFIG, std::string("'") + name + "' is not a valid prepostprocessor.") : r;
}

}  // extern "C"
