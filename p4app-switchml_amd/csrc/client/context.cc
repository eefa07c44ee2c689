// context.cc — see context.h (reference: client_lib/src/context.cc:38-205).
#include "context.h"

#include <hip/hip_runtime_api.h>

#include <cstdio>

#include "loopback_backend.h"

namespace switchml {

void Stats::Init(int n) {
    n_ = n;
    slices_.reset(new std::atomic<uint64_t>[n]);
    ltus_.reset(new std::atomic<uint64_t>[n]);
    bytes_.reset(new std::atomic<uint64_t>[n]);
    ResetStats();
}

void Stats::ResetStats() {
    jobs_submitted_ = 0;
    jobs_finished_ = 0;
    numel_submitted_ = 0;
    for (int i = 0; i < n_; i++) slices_[i] = ltus_[i] = bytes_[i] = 0;
}

void Stats::AddSlice(WorkerTid tid, uint64_t ltus, uint64_t bytes) {
    if (tid < 0 || tid >= n_) return;
    slices_[tid]++;
    ltus_[tid] += ltus;
    bytes_[tid] += bytes;
}

uint64_t Stats::ltus_processed() const {
    uint64_t s = 0;
    for (int i = 0; i < n_; i++) s += ltus_[i];
    return s;
}

uint64_t Stats::slices_processed() const {
    uint64_t s = 0;
    for (int i = 0; i < n_; i++) s += slices_[i];
    return s;
}

void Stats::LogStats() const {
    fprintf(stderr, "[switchml] stats: jobs submitted %llu finished %llu numel %llu\n",
            (unsigned long long)jobs_submitted_.load(), (unsigned long long)jobs_finished_.load(),
            (unsigned long long)numel_submitted_.load());
    for (int i = 0; i < n_; i++)
        fprintf(stderr, "[switchml]   worker thread %d: slices %llu packets %llu bytes %llu\n", i,
                (unsigned long long)slices_[i].load(), (unsigned long long)ltus_[i].load(),
                (unsigned long long)bytes_[i].load());
}

Context& Context::GetInstance() {
    static Context instance;
    return instance;
}

Context::Context() : context_state_(CREATED) {}

Context::~Context() {
    if (context_state_ == RUNNING) Stop();
}

bool Context::Start(Config* config) {
    std::unique_lock<std::mutex> lock(access_mutex_);
    ContextState s = context_state_.load();
    if (s != CREATED && s != STOPPED) return false;
    context_state_ = STARTING;
    try {
        if (config == nullptr) {
            if (!config_.LoadFromFile()) throw SwitchMLFatal("could not start the context: no configuration file");
        } else {
            config_ = *config;
        }
        config_.Validate();
        if (config_.general_.prepostprocessor != "bypass") {
            if (config_.backend_.hip.device >= 0) {
                device_ = config_.backend_.hip.device;
            } else if (hipGetDevice(&device_) != hipSuccess) {
                throw SwitchMLFatal("no HIP device available for the GPU pre/post-processor");
            }
        }
    } catch (...) {
        context_state_ = CREATED;
        throw;
    }
    stats_.Init(config_.general_.num_worker_threads);
    scheduler_.reset(new FifoScheduler(config_));
    backend_.reset(new LoopbackBackend(*this, config_));
    number_of_current_jobs_ = 0;
    context_state_ = RUNNING;  // before the workers start, or they exit at once
    try {
        backend_->SetupWorker();
    } catch (...) {
        context_state_ = STOPPING;
        scheduler_->Stop();
        backend_->CleanupWorker();
        backend_.reset();
        scheduler_.reset();
        context_state_ = CREATED;
        throw;
    }
    return true;
}

void Context::Stop() {
    std::unique_lock<std::mutex> lock(access_mutex_);
    if (context_state_ != RUNNING) throw SwitchMLFatal("the context can only be stopped while RUNNING");
    context_state_ = STOPPING;
    scheduler_->Stop();
    number_of_current_jobs_ = 0;
    lock.unlock();
    backend_->CleanupWorker();  // joins; workers see STOPPING and exit
    lock.lock();
    backend_.reset();
    scheduler_.reset();
    context_state_ = STOPPED;
    lock.unlock();
    all_jobs_finished_event_.notify_all();
}

std::shared_ptr<Job> Context::AllReduceAsync(void* in_ptr, void* out_ptr, uint64_t numel, DataType data_type,
                                             AllReduceOperation op) {
    if (context_state_ != RUNNING) throw SwitchMLFatal("jobs can only be submitted while the context is RUNNING");
    Tensor t;
    t.in_ptr = in_ptr;
    t.out_ptr = out_ptr;
    t.numel = numel;
    t.data_type = data_type;
    ExtraJobInfo extra;
    extra.allreduce_operation = op;
    auto job = std::make_shared<Job>(t, ALLREDUCE, extra);
    {
        std::unique_lock<std::mutex> lock(access_mutex_);
        number_of_current_jobs_++;
    }
    if (!scheduler_->EnqueueJob(job)) {
        std::unique_lock<std::mutex> lock(access_mutex_);
        number_of_current_jobs_--;
    }
    stats_.IncJobsSubmitted(numel);
    return job;
}

std::shared_ptr<Job> Context::AllReduce(void* in_ptr, void* out_ptr, uint64_t numel, DataType data_type,
                                        AllReduceOperation op) {
    auto job = AllReduceAsync(in_ptr, out_ptr, numel, data_type, op);
    job->WaitToComplete();
    return job;
}

void Context::WaitForAllJobs() {
    if (context_state_ != RUNNING) throw SwitchMLFatal("WaitForAllJobs needs a RUNNING context");
    std::unique_lock<std::mutex> lock(access_mutex_);
    all_jobs_finished_event_.wait(lock, [this] { return number_of_current_jobs_ == 0 || context_state_ != RUNNING; });
}

bool Context::GetJobSlice(WorkerTid tid, JobSlice& job_slice) {
    if (context_state_ != RUNNING) return false;
    return scheduler_->GetJobSlice(tid, job_slice);
}

bool Context::GetJobs(size_t max_jobs, std::vector<std::shared_ptr<Job>>& jobs) {
    if (context_state_ != RUNNING) return false;
    return scheduler_->GetJobs(max_jobs, jobs);
}

void Context::NotifyJobSliceCompletion(WorkerTid tid, const JobSlice& job_slice, bool ok) {
    if (!ok) job_slice.job->MarkFailed();
    if (!scheduler_->NotifyJobSliceCompletion(tid, job_slice)) return;
    // The job's last running slice: only now is nothing touching its buffers,
    // so only now may WaitToComplete / sml_job_wait return (FINISHED or FAILED).
    job_slice.job->SetJobStatus(job_slice.job->HasFailed() ? FAILED : FINISHED);
    std::unique_lock<std::mutex> lock(access_mutex_);
    if (number_of_current_jobs_ > 0) number_of_current_jobs_--;
    stats_.IncJobsFinished();
    if (number_of_current_jobs_ == 0) {
        lock.unlock();
        all_jobs_finished_event_.notify_all();
    }
}

}  // namespace switchml
