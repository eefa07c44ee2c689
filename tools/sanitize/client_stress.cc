// client_stress.cc — host-only stress of the client's threading (Context,
// FifoScheduler, Job waits, loopback worker threads) under ThreadSanitizer /
// AddressSanitizer.  Uses the bypass pre/post-processor, so no GPU call is
// made.  Several submitter threads post jobs of ragged sizes concurrently,
// wait on some, WaitForAllJobs, then Stop/Start cycles.  Built and run by
// tools/sanitize/run.sh (not part of the product library).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "context.h"

int main() {
    using namespace switchml;
    for (int cycle = 0; cycle < 3; cycle++) {
        Config cfg;
        const std::string ini =
            "[general]\nnum_workers = 2\nnum_worker_threads = " + std::to_string(1 + cycle * 2) +
            "\nmax_outstanding_packets = 64\npacket_numel = 64\nprepostprocessor = bypass\nbackend = dummy\n"
            "[backend.dummy]\nbandwidth = 0\n";
        cfg.LoadFromString(ini);
        Context& ctx = Context::GetInstance();
        if (!ctx.Start(&cfg)) { fprintf(stderr, "start failed\n"); return 1; }
        std::vector<float> buf(1 << 16, 1.0f);
        std::atomic<int> finished{0};
        std::vector<std::thread> subs;
        for (int s = 0; s < 4; s++) {
            subs.emplace_back([&, s] {
                for (int j = 0; j < 200; j++) {
                    const uint64_t n = 1 + (uint64_t)((j * 7919 + s * 104729) % (1 << 16));
                    auto job = ctx.AllReduceAsync(buf.data(), buf.data(), n, FLOAT32, SUM);
                    if (j % 3 == 0) {
                        job->WaitToComplete();
                        if (job->GetJobStatus() == FINISHED) finished++;
                    }
                }
            });
        }
        for (auto& t : subs) t.join();
        ctx.WaitForAllJobs();
        ctx.Stop();
        printf("cycle %d: waited jobs finished %d\n", cycle, finished.load());
        if (finished.load() != 4 * 67) return 2;
    }
    printf("client stress ok\n");
    return 0;
}
