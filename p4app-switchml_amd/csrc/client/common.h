// common.h — value types of the SwitchML client API, MI355X build.
//
// Mirrors the names and meaning of client_lib/src/common.h:35-116 and
// job.h:36-70 (reference paths relative to /root/reference/dev_root/) so code
// written against the reference compiles unchanged against this header.
// Tensor pointers may be HOST or DEVICE memory: the loopback backend detects
// which (hipPointerGetAttributes) and stages host tensors through HBM.
#ifndef SWITCHML_AMD_COMMON_H_
#define SWITCHML_AMD_COMMON_H_

#include <chrono>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace switchml {

typedef uint64_t JobId;
typedef int16_t WorkerTid;
typedef uint64_t Numel;
typedef std::chrono::steady_clock clock;

// common.h:51-55
enum DataType { FLOAT32, INT32 };

// job.h:36-39 / 44-46
enum JobType { ALLREDUCE, BROADCAST };
enum AllReduceOperation { SUM };
union ExtraJobInfo {
    AllReduceOperation allreduce_operation;
    int32_t broadcast_root_rank;
};

// The reference aborts with LOG(FATAL) on these conditions; this build throws
// (the C-ABI wrappers convert it to an error code).
class SwitchMLFatal : public std::runtime_error {
  public:
    explicit SwitchMLFatal(const std::string& what) : std::runtime_error(what) {}
};

// common.h:62-70
inline uint16_t DataTypeSize(DataType type) {
    if (type == FLOAT32 || type == INT32) return 4;
    throw SwitchMLFatal("'" + std::to_string((int)type) + "' is not a valid tensor data type");
}

// common.h:75-116: a borrowed view of the caller's input/output memory.
struct Tensor {
    void* in_ptr;
    void* out_ptr;
    Numel numel;
    DataType data_type;

    // Advance both pointers by `numel` ELEMENTS of data_type; numel untouched.
    void OffsetPtrs(Numel n) {
        const Numel bytes = n * DataTypeSize(data_type);
        in_ptr = static_cast<char*>(in_ptr) + bytes;
        out_ptr = static_cast<char*>(out_ptr) + bytes;
    }
};

// How long a waiter polls before it sleeps (job completion, a worker's
// stream, an idle worker waiting for the next job), in microseconds.
// SWITCHML_SPIN_US overrides the default; 0 = always sleep at once.
int SpinMicros();

}  // namespace switchml

#endif  // SWITCHML_AMD_COMMON_H_
