#!/bin/bash
# Host-code sanitizers over the client (CPU only; GPU sanitizers are not
# available on this pool).  Usage: tools/sanitize/run.sh [thread|address]
set -euo pipefail
SAN=${1:-thread}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
C=$ROOT/p4app-switchml_amd/csrc/client
OUT=$(mktemp -d)
SRCS="$C/context.cc $C/fifo_scheduler.cc $C/job.cc $C/config.cc $C/loopback_backend.cc $C/hip_exponent_quantizer_ppp.cc $C/xgmi_switch.cc"
g++ -std=c++17 -O1 -g -fsanitize=$SAN -fno-omit-frame-pointer -D__HIP_PLATFORM_AMD__ \
    -I/opt/rocm/include -I$ROOT/include -I$C -o $OUT/client_stress \
    $ROOT/tools/sanitize/client_stress.cc $SRCS \
    -L$ROOT/p4app-switchml_amd/switchml_amd -lswitchml_hip -Wl,-rpath,$ROOT/p4app-switchml_amd/switchml_amd \
    -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -lpthread
"$OUT/client_stress"
