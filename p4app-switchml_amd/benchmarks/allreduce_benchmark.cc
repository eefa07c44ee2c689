// allreduce_benchmark — the reference's AllReduce benchmark CLI
// (dev_root/benchmarks/allreduce_benchmark/main.cc) on the MI355X client:
// same options, data generators, timing loop, verification formula and
// output lines, so scripts written for the reference run unchanged.
// Options take "--name value" or "--name=value"; booleans accept true/false/1/0.
// Extra options of this build: --config <switchml.cfg> (else the reference's
// search path, else general.cfg-like defaults), --mode bulk|fused|packet,
// --num-workers N, --num-worker-threads T, --packet-numel P, --bandwidth Mbps.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <iostream>
#include <limits>
#include <map>
#include <numeric>
#include <string>
#include <vector>

#include "context.h"

namespace {

struct Opts {
    uint64_t tensor_numel = 268435456;   // main.cc:101
    std::string tensor_type = "int32";
    std::string device = "cpu";
    uint32_t num_jobs = 10;
    uint32_t num_warmup = 5;
    bool inplace = true;
    bool verify = false;
    uint32_t sync_every = 1;
    float err = 1.0f;
    bool random = false;
    uint32_t seed = 0;
    bool dump_stats = false;
    std::string config;
    std::map<std::string, std::string> overrides;
};

bool to_bool(const std::string& v) { return v == "true" || v == "1" || v == "yes" || v == "on"; }

void usage() {
    std::cout << "Allreduce Test:\n"
                 "  -h [ --help ]                      Display this help message\n"
                 "  --tensor-numel arg (=268435456)    Number of elements to all reduce.\n"
                 "  --tensor-type arg (=int32)         Specify the data type to use. Choose from [float, int32].\n"
                 "  --device arg (=cpu)                Allocate the tensors on the specified device. Choose from [cpu, gpu]\n"
                 "  --num-jobs arg (=10)               How many timed all reduce jobs should we submit?\n"
                 "  --num-warmup-jobs arg (=5)         How many untimed all reduce jobs should we submit before the timed ones?\n"
                 "  --inplace arg (=1)                 Use the same memory region as source and destination?\n"
                 "  --verify arg (=0)                  Verify results to make sure they are as expected\n"
                 "  --sync-every arg (=1)              When to wait for the submitted jobs (0 = only after all).\n"
                 "  --err arg (=1)                     The allowed error percentage. Used when verify is set to true\n"
                 "  --random arg (=0)                  Initialize the data with random values.\n"
                 "  --seed arg (=0)                    Random seed (0 = time).\n"
                 "  --dump-stats arg (=0)              Print and clear the switchml statistics after each sync?\n"
                 "  --config arg                       switchml.cfg to use (MI355X build)\n"
                 "  --mode / --num-workers / --num-worker-threads / --packet-numel / --bandwidth / --batch-jobs\n"
                 "                                     config overrides (MI355X build)\n";
}

Opts parse(int argc, char** argv) {
    Opts o;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i], v;
        if (a == "-h" || a == "--help") {
            usage();
            exit(EXIT_SUCCESS);
        }
        if (a.rfind("--", 0) != 0) {
            std::cerr << "unexpected argument '" << a << "'\n";
            exit(EXIT_FAILURE);
        }
        auto eq = a.find('=');
        if (eq != std::string::npos) {
            v = a.substr(eq + 1);
            a = a.substr(0, eq);
        } else if (i + 1 < argc) {
            v = argv[++i];
        } else {
            std::cerr << "missing value for " << a << "\n";
            exit(EXIT_FAILURE);
        }
        if (a == "--tensor-numel") o.tensor_numel = std::stoull(v);
        else if (a == "--tensor-type") o.tensor_type = v;
        else if (a == "--device") o.device = v;
        else if (a == "--num-jobs") o.num_jobs = std::stoul(v);
        else if (a == "--num-warmup-jobs") o.num_warmup = std::stoul(v);
        else if (a == "--inplace") o.inplace = to_bool(v);
        else if (a == "--verify") o.verify = to_bool(v);
        else if (a == "--sync-every") o.sync_every = std::stoul(v);
        else if (a == "--err") o.err = std::stof(v);
        else if (a == "--random") o.random = to_bool(v);
        else if (a == "--seed") o.seed = std::stoul(v);
        else if (a == "--dump-stats") o.dump_stats = to_bool(v);
        else if (a == "--config") o.config = v;
        else if (a == "--mode") o.overrides["backend.hip.mode"] = v;
        else if (a == "--num-workers") o.overrides["general.num_workers"] = v;
        else if (a == "--num-worker-threads") o.overrides["general.num_worker_threads"] = v;
        else if (a == "--packet-numel") o.overrides["general.packet_numel"] = v;
        else if (a == "--bandwidth") o.overrides["backend.dummy.bandwidth"] = v;
        else if (a == "--batch-jobs") o.overrides["backend.hip.batch_jobs"] = v;
        else {
            std::cerr << "unrecognised option '" << a << "'\n";
            exit(EXIT_FAILURE);
        }
    }
    if (o.sync_every == 0) o.sync_every = o.num_jobs;
    return o;
}

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        std::cerr << what << ": " << hipGetErrorString(e) << "\n";
        exit(EXIT_FAILURE);
    }
}

}  // namespace

int main(int argc, char** argv) {
    Opts o = parse(argc, argv);
    switchml::Config cfg;
    // general.cfg / dummy.cfg shipped values as the fallback configuration
    cfg.general_.packet_numel = 256;
    cfg.backend_.dummy.bandwidth = 100000.0f;
    if (!o.config.empty()) {
        if (!cfg.LoadFromFile(o.config)) {
            std::cerr << "cannot read config '" << o.config << "'\n";
            return EXIT_FAILURE;
        }
    } else {
        cfg.LoadFromFile();  // optional
    }
    std::string extra;
    for (auto& kv : o.overrides) {
        auto dot = kv.first.rfind('.');
        extra += "[" + kv.first.substr(0, dot) + "]\n" + kv.first.substr(dot + 1) + " = " + kv.second + "\n";
    }
    cfg.LoadFromString(extra);

    switchml::Context& ctx = switchml::Context::GetInstance();
    ctx.Start(&cfg);
    const uint16_t W = ctx.GetConfig().general_.num_workers;

    if (o.random) {
        if (o.seed == 0) o.seed = (uint32_t)time(NULL);
        srand(o.seed);
        std::cout << "Using random seed " << o.seed << std::endl;
    }
    const bool is_float = o.tensor_type == "float";
    if (!is_float && o.tensor_type != "int32") {
        std::cout << "'" << o.tensor_type << "' is not a valid tensor type. Choose from [float, int32]" << std::endl;
        return EXIT_FAILURE;
    }
    const switchml::DataType dt = is_float ? switchml::FLOAT32 : switchml::INT32;
    const size_t bytes = o.tensor_numel * 4;
    std::vector<uint32_t> src(o.tensor_numel), ctrl;
    std::vector<uint32_t> dst(o.inplace ? 0 : o.tensor_numel);
    // data generators: main.cc:189-251
    for (uint64_t i = 0; i < o.tensor_numel; i++) {
        if (is_float) {
            float f;
            if (o.random) {
                int r = rand();
                int bits = ((r % 2) << 31) | ((r % 254) << 23) | (r % (1 << 23));
                memcpy(&f, &bits, 4);
            } else {
                f = float(i) * ((i % 2) ? -1.0f : 1.0f);
            }
            memcpy(&src[i], &f, 4);
        } else {
            int32_t v = o.random ? (int32_t)((uint32_t)rand() + (uint32_t)rand())
                                 : (int32_t)((uint32_t)i * ((i % 2) ? 0xffffffffu : 1u));
            src[i] = (uint32_t)v;
        }
    }
    if (!o.inplace) {
        for (auto& d : dst) {
            if (is_float) {
                float f = (float)123456789;  // main.cc:219 stores 123456789 into a float
                memcpy(&d, &f, 4);
            } else {
                d = 123456789;
            }
        }
    }
    ctrl = src;

    void* src_data = src.data();
    void* dst_data = o.inplace ? src.data() : dst.data();
    void *gsrc = nullptr, *gdst = nullptr;
    if (o.device == "gpu") {
        hip_check(hipMalloc(&gsrc, bytes), "hipMalloc");
        hip_check(hipMemcpy(gsrc, src.data(), bytes, hipMemcpyHostToDevice), "hipMemcpy");
        if (o.inplace) {
            gdst = gsrc;
        } else {
            hip_check(hipMalloc(&gdst, bytes), "hipMalloc");
            hip_check(hipMemcpy(gdst, dst.data(), bytes, hipMemcpyHostToDevice), "hipMemcpy");
        }
        src_data = gsrc;
        dst_data = gdst;
    } else if (o.device != "cpu") {
        std::cout << "'" << o.device << "' is not a valid device. Choose from [cpu, gpu]" << std::endl;
        return EXIT_FAILURE;
    }

    std::cout << "Submitting " << o.num_warmup << " warmup jobs." << std::endl;
    for (uint32_t i = 0; i < o.num_warmup; i++) ctx.AllReduceAsync(src_data, dst_data, o.tensor_numel, dt, switchml::SUM);
    ctx.WaitForAllJobs();
    std::cout << "Warmup finished." << std::endl;

    std::cout << "Submitting " << o.num_jobs << " jobs." << std::endl;
    std::vector<unsigned long> durations_ns;
    auto begin = switchml::clock::now();
    uint32_t jobs_before_sync = 0;
    for (uint32_t i = 0; i < o.num_jobs; i++) {
        ctx.AllReduceAsync(src_data, dst_data, o.tensor_numel, dt, switchml::SUM);
        jobs_before_sync++;
        if ((i + 1) % o.sync_every == 0) {
            ctx.WaitForAllJobs();
            durations_ns.push_back(
                std::chrono::duration_cast<std::chrono::nanoseconds>(switchml::clock::now() - begin).count());
            char job_str[40];
            if (jobs_before_sync > 1) snprintf(job_str, sizeof(job_str), "%u-%u", i - jobs_before_sync + 1, i);
            else snprintf(job_str, sizeof(job_str), "%u", i);
            std::cout << "Job(s) #" << job_str << "# finished. Duration: #" << durations_ns.back()
                      << "# ns Goodput: #" << o.tensor_numel * 4.0 * 8 * jobs_before_sync / durations_ns.back()
                      << "# Gbps." << std::endl;
            jobs_before_sync = 0;
            if (o.dump_stats) {
                ctx.GetStats().LogStats();
                ctx.GetStats().ResetStats();
            }
            begin = switchml::clock::now();
        }
    }
    ctx.WaitForAllJobs();
    std::cout << "All jobs finished." << std::endl;

    if (o.verify) {
        std::cout << "Verifying final results" << std::endl;
        if (o.device == "gpu") {
            hip_check(hipMemcpy(src.data(), gsrc, bytes, hipMemcpyDeviceToHost), "hipMemcpy");
            if (!o.inplace) hip_check(hipMemcpy(dst.data(), gdst, bytes, hipMemcpyDeviceToHost), "hipMemcpy");
        }
        const uint32_t* out = o.inplace ? src.data() : dst.data();
        int max_num_errors = 10;
        // main.cc:343: in place, the tensor was reduced num_jobs + num_warmup times
        const double mult = o.inplace ? std::pow((double)W, o.num_jobs + o.num_warmup) : (double)W;
        for (uint64_t j = 0; j < o.tensor_numel && max_num_errors > 0; j++) {
            if (is_float) {
                float ein, eout, got;
                memcpy(&ein, &ctrl[j], 4);
                memcpy(&got, &out[j], 4);
                eout = ein * (float)mult;
                float error = (eout - got) / eout * 100;   // signed, as main.cc:347
                if (error > o.err) {
                    printf("Verification error at output buffer index [%lu]. Expected %e but found %e (%.2f%% error).\n",
                           (unsigned long)j, eout, got, error);
                    max_num_errors--;
                }
                if (!o.inplace) {  // main.cc:361-367: the input buffer must be left untouched
                    float in;
                    memcpy(&in, &src[j], 4);
                    error = (ein - in) / (ein + std::numeric_limits<float>::epsilon()) * 100;
                    if (error > o.err) {
                        printf("Verification error at input buffer index [%lu]. Expected %e but found %e (%.2f%% error).\n",
                               (unsigned long)j, ein, in, error);
                        max_num_errors--;
                    }
                }
            } else {
                int32_t ein = (int32_t)ctrl[j], got = (int32_t)out[j];
                int32_t eout = (int32_t)((uint32_t)ein * (uint32_t)(int64_t)mult);
                float error = (eout - got) / float(eout) * 100;
                if (error > o.err) {
                    printf("Verification error at output buffer index [%lu]. Expected %d but found %d (%.2f%% error).\n",
                           (unsigned long)j, eout, got, error);
                    max_num_errors--;
                }
                if (!o.inplace) {  // main.cc:385-391
                    const int32_t in = (int32_t)src[j];
                    error = (ein - in) / (float(ein) + std::numeric_limits<float>::epsilon()) * 100;
                    if (error > o.err) {
                        printf("Verification error at input buffer index [%lu]. Expected %d but found %d (%.2f%% error).\n",
                               (unsigned long)j, ein, in, error);
                        max_num_errors--;
                    }
                }
            }
        }
        if (max_num_errors == 10) std::cout << "Data verified successfully." << std::endl;
        else std::cout << "Verification failed. There could be more errors but we do not print more than 10." << std::endl;
    }

    const double num_bits = (double)o.sync_every * o.tensor_numel * 4 * 8;
    std::cout << std::endl << std::endl;
    uint64_t mn = *std::min_element(durations_ns.begin(), durations_ns.end());
    std::cout << "Min " << mn << " ns " << num_bits / mn << " Gbps" << std::endl;
    uint64_t mx = *std::max_element(durations_ns.begin(), durations_ns.end());
    std::cout << "Max " << mx << " ns " << num_bits / mx << " Gbps" << std::endl;
    std::vector<unsigned long> sorted = durations_ns;
    std::nth_element(sorted.begin(), sorted.begin() + sorted.size() / 2, sorted.end());
    uint64_t med = sorted[sorted.size() / 2];
    std::cout << "Median " << med << " ns " << num_bits / med << " Gbps" << std::endl;
    double mean = std::accumulate(durations_ns.begin(), durations_ns.end(), 0.0) / durations_ns.size();
    std::cout << "Mean " << (uint64_t)mean << " ns " << num_bits / mean << " Gbps" << std::endl;
    double sq = 0;
    for (auto d : durations_ns) sq += (d - mean) * (d - mean);
    std::cout << "Std dev " << std::sqrt(sq / durations_ns.size()) << " ns" << std::endl;

    std::cout << "Cleaning up." << std::endl;
    ctx.Stop();
    if (gsrc) (void)hipFree(gsrc);
    if (gdst && gdst != gsrc) (void)hipFree(gdst);
    return EXIT_SUCCESS;
}
