#!/usr/bin/env python3
"""Static evidence for DESIGN.md §9 F2: which collective algorithms the
installed RCCL has DEVICE code for.  RCCL names every device function
ncclDevFunc_<Collective>_<ALGO>_<PROTO>_<RedOp>_<type>_...; a CollNet
all-reduce needs ncclDevFunc_AllReduce_COLLNET_DIRECT_* / _COLLNET_CHAIN_*
functions, without which no CollNet plugin can ever be handed an all-reduce.

Usage: python tools/rccl_devfuncs.py [librccl.so] [OUT.json]"""
import collections
import json
import os
import re
import sys


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else "/opt/rocm/lib/librccl.so"
    path = os.path.realpath(lib)
    with open(path, "rb") as f:
        data = f.read()
    names = sorted(set(m.group().decode() for m in re.finditer(rb"ncclDevFunc_[A-Za-z0-9_]+", data)))
    per = collections.Counter()
    for n in names:
        p = n.split("_")
        per[f"{p[1]}/{p[2]}"] += 1
    allreduce_algos = sorted({n.split("_")[2] for n in names if n.startswith("ncclDevFunc_AllReduce_")})
    out = {
        "library": path,
        "device_functions": len(names),
        "per_collective_and_algorithm": dict(sorted(per.items())),
        "allreduce_algorithms_with_device_code": allreduce_algos,
        "collnet_allreduce_device_functions": [n for n in names if "COLLNET" in n],
        "finding": ("no ncclDevFunc_AllReduce_COLLNET_DIRECT_* / _COLLNET_CHAIN_* device function exists: "
                    "this RCCL cannot run a CollNet all-reduce, whatever plugin is loaded"
                    if not any("COLLNET" in n for n in names) else "CollNet device functions present"),
    }
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
