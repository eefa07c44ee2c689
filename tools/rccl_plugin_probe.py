#!/usr/bin/env python3
"""Does RCCL itself load the SwitchML CollNet plugin?  One rank per process,
NCCL_NET_PLUGIN = librccl-net-switchml.so, NCCL_COLLNET_ENABLE=1, RCCL's own
INIT/NET log captured, one all_reduce.  Prints the plugin-related log lines
and whether the all_reduce was correct.  (A CollNet all-reduce proper needs
several nodes; this checks the loading / symbol / init handshake.)

Usage: python tools/rccl_plugin_probe.py [world_size]   (spawns the ranks)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PLUGIN = os.path.join(ROOT, "p4app-switchml_amd", "switchml_amd", "librccl-net-switchml.so")


def rank_main(rank, world, port):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "p4app-switchml_amd")]
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            device_id=torch.device("cuda:0"))
    x = torch.full((1 << 20,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    ok = bool((x == world * (world + 1) / 2).all())
    dist.destroy_process_group()
    print(json.dumps({"rank": rank, "allreduce_ok": ok}), flush=True)


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[1] == "--rank":
    rank_main(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
elif __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    out_dir = os.path.join(ROOT, "gpurun_out", "rccl_probe")
    os.makedirs(out_dir, exist_ok=True)
    ini = ("[general]\nnum_workers = %d\nnum_worker_threads = 2\nprepostprocessor = hip_exponent_quantizer\n"
           "[backend.dummy]\nbandwidth = 0\n[backend.hip]\ndevice = 0\n" % world)
    env = dict(os.environ, NCCL_NET_PLUGIN=PLUGIN, NCCL_COLLNET_ENABLE="1", NCCL_DEBUG="INFO",
               SWITCHML_COLLNET_LOOPBACK="1",
               NCCL_DEBUG_SUBSYS="INIT,NET,ENV", NCCL_DEBUG_FILE=os.path.join(out_dir, "rccl.%p.log"),
               SWITCHML_CONFIG_INI=ini)
    port = 29611
    procs = [subprocess.Popen([sys.executable, __file__, "--rank", str(r), str(world), str(port)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = [p.communicate(timeout=240)[0] for p in procs]
    lines = []
    for f in sorted(os.listdir(out_dir)):
        with open(os.path.join(out_dir, f), errors="replace") as fh:
            lines += [l.rstrip() for l in fh if any(k in l for k in ("Plugin", "plugin", "SWITCHML", "SwitchML",
                                                                      "CollNet", "collnet", "NET/"))]
    print(json.dumps({"returncodes": [p.returncode for p in procs],
                      "rank_output": [o.strip().splitlines()[-3:] for o in outs],
                      "rccl_plugin_log": lines[:40]}, indent=1))
