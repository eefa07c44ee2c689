// hello_world — dev_root/examples/hello_world/main.cc on the MI355X client:
// 8 asynchronous float AllReduces of 2^15 elements through the Context, then
// out == in * num_workers within 1 % (signed) and the input unchanged.
// Usage: hello_world [switchml.cfg]   (default: the reference's search path,
// else general.cfg values with the loopback backend).
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <vector>

#include "context.h"

int main(int argc, char** argv) {
    switchml::Context& ctx = switchml::Context::GetInstance();
    printf("Hello world!. Starting the switchml context\n");
    switchml::Config cfg;
    cfg.general_.packet_numel = 256;
    cfg.backend_.dummy.bandwidth = 0;
    if (argc > 1) {
        if (!cfg.LoadFromFile(argv[1])) {
            fprintf(stderr, "cannot read %s\n", argv[1]);
            return 1;
        }
    } else {
        cfg.LoadFromFile();
    }
    ctx.Start(&cfg);

    const uint64_t numel = 1 << 15;
    const int num_tensors = 8;
    const int num_workers = ctx.GetConfig().general_.num_workers;
    std::vector<std::vector<float>> in(num_tensors, std::vector<float>(numel)), out = in;
    for (int i = 0; i < num_tensors; i++)
        for (uint64_t j = 0; j < numel; j++) in[i][j] = i * numel + j;

    printf("Submitting all reduce jobs\n");
    for (int i = 0; i < num_tensors; i++)
        ctx.AllReduceAsync(in[i].data(), out[i].data(), numel, switchml::FLOAT32, switchml::SUM);
    printf("Waiting for all jobs to finish\n");
    ctx.WaitForAllJobs();
    printf("Stopping the switchml context\n");
    ctx.Stop();

    printf("Verifying results\n");
    for (int i = 0; i < num_tensors; i++) {
        for (uint64_t j = 0; j < numel; j++) {
            float input = i * numel + j;
            float expected = input * num_workers;
            float error = (expected - out[i][j]) / (expected + std::numeric_limits<float>::epsilon()) * 100;
            if (error > 1) {
                printf("Failed to verify output data. Element %lu in tensor %d was %e but we expected %e (error %.2f%%)\n",
                       (unsigned long)j, i, out[i][j], expected, error);
                return 1;
            }
            if (in[i][j] != input) {
                printf("Failed to verify that input data is unchanged. Element %lu in tensor %d\n", (unsigned long)j, i);
                return 1;
            }
        }
    }
    printf("Data verified successfully exiting main program\n");
    return 0;
}
