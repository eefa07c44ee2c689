// job.cc — Job lifecycle (client_lib/src/job.cc).
#include "job.h"

namespace switchml {

std::atomic<JobId> Job::next_id_{0};

Job::Job(Tensor tensor, JobType job_type, ExtraJobInfo extra_job_info)
    : id_(next_id_++), tensor_(tensor), job_type_(job_type), extra_job_info_(extra_job_info), job_status_(INIT) {}

void Job::WaitToComplete() {
    std::unique_lock<std::mutex> lock(access_mutex_);
    job_finished_event_.wait(lock, [this] {
        JobStatus s = job_status_.load();
        return s == FINISHED || s == FAILED;
    });
}

void Job::SetJobStatus(JobStatus status) {
    std::unique_lock<std::mutex> lock(access_mutex_);
    if (status < job_status_.load()) return;  // never move backwards
    job_status_.store(status);
    if (status == FINISHED || status == FAILED) {
        lock.unlock();
        job_finished_event_.notify_all();
    }
}

}  // namespace switchml
