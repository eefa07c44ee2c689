// job.cc — Job lifecycle (client_lib/src/job.cc).
#include "job.h"

#include <chrono>
#include <cstdlib>
#include <thread>

namespace switchml {

std::atomic<JobId> Job::next_id_{0};

int SpinMicros() {
    static const int us = [] {
        const char* e = std::getenv("SWITCHML_SPIN_US");
        if (!e || !*e) return 300;
        const int v = std::atoi(e);
        return v < 0 ? 0 : v;
    }();
    return us;
}

Job::Job(Tensor tensor, JobType job_type, ExtraJobInfo extra_job_info)
    : id_(next_id_++), tensor_(tensor), job_type_(job_type), extra_job_info_(extra_job_info), job_status_(INIT) {}

void Job::WaitToComplete() {
    // GPU jobs finish in tens of microseconds: poll briefly before sleeping on
    // the condition variable (a futex wake-up costs about as much as the job).
    const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(SpinMicros());
    do {
        const JobStatus s = job_status_.load(std::memory_order_acquire);
        if (s == FINISHED || s == FAILED) return;
        std::this_thread::yield();
    } while (std::chrono::steady_clock::now() < until);
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
