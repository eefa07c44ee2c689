"""RCCL with the SwitchML plugin library, for real: W worker processes,
torch.distributed backend "nccl" (= RCCL), NCCL_NET_PLUGIN =
librccl-net-switchml.so, NCCL_COLLNET_ENABLE=1.

The reference's integration (frameworks_integration/nccl_plugin) is a
CollNet plugin NCCL calls for an all-reduce across nodes (each node's head
rank hands its buffer to `iallreduce`, the switch sums the nodes' data,
switchml_plugin.cc:293-387), paired with a p2p net table.  Here:

* NCCL_HOSTID = a distinct id per rank, so every rank is a CollNet "node"
  of its own — the way each SwitchML worker is a host with a NIC to the
  switch.  On an 8-GPU node the ranks use GPUs 0..W-1; on a one-GPU box
  (`same_gpu`) they share cuda:0 (two ranks of one host on one device are
  refused by RCCL, two hosts' ranks are not);
* RCCL's p2p traffic runs over the library's own TCP net
  (plugins/rccl_collnet/socket_net.h): RCCL loads both tables and keeps the
  CollNet one only because that net works;
* the CollNet table DECLINES RCCL by default (switchml_collnet.cc sml_init):
  RCCL 7.2 on MI355X has no working CollNet AllReduce — its tuner picks
  CollNetChain, whose kernels it does not build, and the AllReduce returns
  unreduced; CollNetDirect needs a switch node in the topology and then
  hangs (measured: profiles/r03/rccl_collnet/).  RCCL then logs "Cannot
  initialize CollNet, using point-to-point network instead" and reduces with
  its own algorithms over the SwitchML net — correct results.
  `allow_collnet=True` (SWITCHML_COLLNET_RCCL=1) offers the table anyway,
  with NCCL_ALGO=CollNetDirect and a switch node added to each worker's
  topology (`add_switch_node`): the experiment that shows the hang;
* behind the table (driven by hand, and by RCCL when allowed) is the in-node
  switch (general.backend = xgmi, xgmi_switch.h); the plugin keeps the W
  workers' submission order identical (job_order.h).

Each rank reports the plugin's call counters (`switchml_collnet_stats`),
RCCL's all-reduce of integer-valued data against the exact sum, the same
buffer through the plugin's iallreduce by hand (the xgmi switch) against it
too, N(0,1) data within the quantization bound, and RCCL all-reduces of
configs[4]'s ResNet-50 buckets.  The parent (`launch`) never touches the GPU.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys
import time
import uuid

_HERE = os.path.dirname(os.path.abspath(__file__))
PLUGIN_PATH = os.path.join(_HERE, "librccl-net-switchml.so")
RESNET50_BUCKETS = [6_553_600, 6_553_600, 6_553_600, 5_896_232]
STATS = ("init", "connect", "iallreduce", "iallreduce_bytes", "test_done", "reg_mr", "iallreduce_submitted",
         "declined")


def collnet_stats(path: str = PLUGIN_PATH) -> dict:
    """The plugin's CollNet call counters in THIS process (RCCL dlopens the
    same file, so this is the instance RCCL calls)."""
    lib = ctypes.CDLL(path)
    buf = (ctypes.c_uint64 * len(STATS))()
    n = lib.switchml_collnet_stats(buf, len(STATS))
    return {k: int(buf[i]) for i, k in enumerate(STATS[:n])}


SAME_GPU_NETS = ("switchml", "socket")


def same_gpu_rccl_env(rank: int, session: str, net: str = "switchml") -> dict:
    """RCCL environment for W ranks that share ONE GPU (a one-GPU box standing
    in for a node): RCCL refuses two ranks of one host on one device, so each
    rank is a host of its own (NCCL_HOSTID), and the ranks reach each other
    through a net — `net` = "switchml": this library's TCP net
    (NCCL_NET_PLUGIN = librccl-net-switchml.so; its CollNet table declines
    RCCL, so only the net is used), "socket": RCCL's built-in socket net over
    the loopback interface.  The reductions (ncclInt8 MAX, ncclInt32 SUM) run
    in RCCL's own ring kernels either way — the code the N-GPU node runs —
    only the transport between the ranks differs.  Set these before
    init_process_group("nccl")."""
    if net not in SAME_GPU_NETS:
        raise ValueError(f"net must be one of {SAME_GPU_NETS}")
    env = {"NCCL_HOSTID": f"switchml-worker-{session}-{rank}", "RCCL_MSCCL_ENABLE": "0",
           "RCCL_MSCCLPP_ENABLE": "0", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    if net == "switchml":
        env["NCCL_NET_PLUGIN"] = PLUGIN_PATH
    else:
        env.update(NCCL_NET_PLUGIN="none", NCCL_NET="Socket", NCCL_SOCKET_IFNAME="lo")
    return env


def rank_env(rank: int, world: int, device: int, session: str, channels: int, algo: str | None,
             log_dir: str | None, threads: int = 1, packet_numel: int = 256) -> dict:
    ini = (f"[general]\nrank = {rank}\nnum_workers = {world}\nnum_worker_threads = {threads}\n"
           f"packet_numel = {packet_numel}\nbackend = xgmi\nprepostprocessor = hip_exponent_quantizer\n"
           f"[backend.xgmi]\nsession = {session}\ntimeout_ms = 120000\n[backend.hip]\ndevice = {device}\n")
    env = {
        "NCCL_NET_PLUGIN": PLUGIN_PATH,
        "NCCL_COLLNET_ENABLE": "1",
        "NCCL_HOSTID": f"switchml-worker-{session}-{rank}",
        "RCCL_MSCCL_ENABLE": "0",
        "RCCL_MSCCLPP_ENABLE": "0",
        "SWITCHML_CONFIG_INI": ini,
        "HSA_ENABLE_IPC_MODE_LEGACY": "0",
    }
    env.pop("SWITCHML_NET_PLUGIN", None)
    if channels > 0:
        env["NCCL_MAX_NCHANNELS"] = str(channels)
    if algo:
        env["NCCL_ALGO"] = algo
    if log_dir:
        env.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,NET,GRAPH,ENV,TUNING",
                   NCCL_DEBUG_FILE=os.path.join(log_dir, f"rccl.rank{rank}.%p.log"))
    return env


def worker_env(parent: dict, rank: int, world: int, device: int, session: str, channels: int = 0,
               algo: str | None = None, log_dir: str | None = None, extra_env: dict | None = None) -> dict:
    """A worker's environment: the parent's, minus what a launcher put there
    for ITS ranks — under torch.distributed.run, TORCHELASTIC_USE_AGENT_STORE
    makes every rank of a tcp:// rendezvous a store client with no server (a
    silent hang), and RANK / WORLD_SIZE / MASTER_* name the wrong group —
    plus rank_env and `extra_env`."""
    env = {k: v for k, v in parent.items()
           if not k.startswith(("TORCHELASTIC_", "ROLE_", "GROUP_"))
           and k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                         "SWITCHML_NET_PLUGIN")}
    env.update(rank_env(rank, world, device, session, channels, algo, log_dir))
    env.update(extra_env or {})
    env["PYTHONPATH"] = os.path.dirname(_HERE) + os.pathsep + env.get("PYTHONPATH", "")
    return env


def _bound(xs, out_ref, world):
    """|out - sum x| <= per-element quantization bound, with the global block
    exponent e (max over workers): each worker rounds to 2^(e-31) * W units
    (half a unit each), the dequantized sum rounds once more (half an ulp)."""
    import numpy as np
    s = np.sum(np.stack(xs).astype(np.float64), axis=0)
    err = np.abs(out_ref.astype(np.float64) - s)
    amax = max(float(np.max(np.abs(x))) for x in xs)
    e = np.floor(np.log2(amax)) + 1 if amax > 0 else 0
    unit = world * 2.0 ** (e - 31)
    lim = world * 0.5 * unit + np.abs(s) * 2.0 ** -23 + unit
    return float(err.max()), bool((err <= lim).all())


def add_switch_node(src: str, dst: str):
    """RCCL topology XML `src` with one link from every GPU to a switch node
    (<xgmi tclass="0x068000">, the NVSwitch PCI class RCCL's topology parser
    turns into an NVS node)."""
    import xml.etree.ElementTree as ET
    tree = ET.parse(src)
    gpus = tree.getroot().findall(".//gpu")
    if not gpus:
        raise RuntimeError(f"no <gpu> in {src}")
    for g in gpus:
        ET.SubElement(g, "xgmi", {"target": "0000:ff:00.0", "count": "1", "tclass": "0x068000"})
    tree.write(dst)


def rank_main(a):
    import numpy as np
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", a.device)
    torch.cuda.set_device(dev)
    # rendezvous: a FileStore the launcher named (no port chosen by one
    # process and bound by another later), or tcp on --port
    inits = ([f"file://{a.init}", f"file://{a.init}.2"] if a.init else
             [f"tcp://127.0.0.1:{a.port}", f"tcp://127.0.0.1:{a.port + 1}"])
    topo = None
    if a.switch_topo:
        # RCCL 7.2 runs AllReduce on CollNet only as CollNetDirect, which its
        # tuner enables only when the topology holds a switch node (it
        # disables CollNetDirect when ncclTopoGetNvsCount() == 0).  Each
        # worker here is a one-GPU CollNet node; a switch node attached to
        # that GPU has no other GPU to route to, so it changes nothing but
        # that check.  RCCL's own detected topology is dumped first (a
        # throwaway communicator), the node added, and the file handed back
        # through NCCL_TOPO_FILE.
        dump = os.path.join(a.topo_dir, f"detected.rank{a.rank}.xml")
        os.environ["NCCL_TOPO_DUMP_FILE"] = dump
        os.environ["NCCL_TOPO_DUMP_FILE_RANK"] = str(a.rank)
        dist.init_process_group("nccl", init_method=inits.pop(0), rank=a.rank, world_size=a.world,
                                device_id=dev)
        dist.destroy_process_group()
        del os.environ["NCCL_TOPO_DUMP_FILE"]
        topo = os.path.join(a.topo_dir, f"with_switch.rank{a.rank}.xml")
        add_switch_node(dump, topo)
        os.environ["NCCL_TOPO_FILE"] = topo
    dist.init_process_group("nccl", init_method=inits[0], rank=a.rank, world_size=a.world,
                            device_id=dev)
    out = {"rank": a.rank, "device": a.device, "topology_file": topo}
    W = a.world
    n = a.numel

    def say(msg):
        print(f"[rank {a.rank}] {msg}", flush=True)

    say("process group up")
    if os.environ.get("SWITCHML_COLLNET_TRACE"):
        import threading

        def watch():
            while True:
                time.sleep(5)
                say(f"collnet stats {collnet_stats()}")
        threading.Thread(target=watch, daemon=True).start()

    def allreduce(t):
        dist.all_reduce(t)
        torch.cuda.synchronize()

    # 1) integer-valued data: every path is exact, so RCCL == exact sum bit for bit
    gens = [np.random.default_rng(1000 + r) for r in range(W)]
    xs = [g.integers(-1000, 1001, n).astype(np.float32) for g in gens]
    exact = np.sum(np.stack(xs), axis=0, dtype=np.float32)
    t = torch.from_numpy(xs[a.rank]).to(dev)
    before = collnet_stats()
    allreduce(t)
    after = collnet_stats()
    out["stats_before"], out["stats_after_first"] = before, after
    say(f"integer all-reduce done, iallreduce calls {after['iallreduce'] - before['iallreduce']}")
    r_int = t.cpu().numpy()
    out["int_exact"] = bool(np.array_equal(r_int.view(np.uint32), exact.view(np.uint32)))

    # the same data through the plugin's iallreduce by hand, on a FRESH copy
    # of this rank's input (not RCCL's output buffer): the xgmi switch, one
    # job.  hand_int_exact checks it against the exact sum on its own;
    # int_equal_direct compares it with RCCL's result — so when RCCL's
    # all-reduce is wrong (CollNetChain's no-op) that one is
    # False while hand_int_exact stays True.
    from .collnet import CollNetComm
    comm = CollNetComm(nranks=W, rank=a.rank, path=PLUGIN_PATH)
    h = torch.from_numpy(xs[a.rank].copy()).to(dev)
    torch.cuda.synchronize()
    comm.wait(comm.iallreduce(h.data_ptr(), h.data_ptr(), n))
    r_hand = h.cpu().numpy()
    out["hand_int_exact"] = bool(np.array_equal(r_hand.view(np.uint32), exact.view(np.uint32)))
    out["int_equal_direct"] = bool(np.array_equal(r_hand.view(np.uint32), r_int.view(np.uint32)))
    say(f"by-hand iallreduce done: RCCL int_exact {out['int_exact']}, by-hand int_exact {out['hand_int_exact']}, "
        f"by-hand equal to RCCL {out['int_equal_direct']}")

    # 2) N(0,1) data: RCCL vs by hand (equal when RCCL's CollNet chunks start
    # on packet boundaries) and vs the fp32 sum within the quantization bound
    ys = [np.random.default_rng(2000 + r).standard_normal(n).astype(np.float32) for r in range(W)]
    t = torch.from_numpy(ys[a.rank]).to(dev)
    allreduce(t)
    r_rccl = t.cpu().numpy()
    h = torch.from_numpy(ys[a.rank]).to(dev)
    torch.cuda.synchronize()
    comm.wait(comm.iallreduce(h.data_ptr(), h.data_ptr(), n))
    r_hand = h.cpu().numpy()
    out["normal_equal_direct"] = bool(np.array_equal(r_hand.view(np.uint32), r_rccl.view(np.uint32)))
    out["normal_max_err"], out["normal_within_bound"] = _bound(ys, r_rccl, W)
    say(f"N(0,1) done: equal_direct {out['normal_equal_direct']} within_bound {out['normal_within_bound']}")
    comm.close()

    # 3) configs[4]: ResNet-50 DDP buckets all-reduced by RCCL (through CollNet)
    if a.iters > 0:
        bk = [torch.randn(m, device=dev) * 1e-3 for m in RESNET50_BUCKETS]
        for b in bk:
            dist.all_reduce(b)
        torch.cuda.synchronize()
        dist.barrier()
        c0 = collnet_stats()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            for b in bk:
                dist.all_reduce(b)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        c1 = collnet_stats()
        out["configs4_ms_per_iter"] = 1e3 * dt / a.iters
        out["configs4_iallreduce_calls_per_iter"] = (c1["iallreduce"] - c0["iallreduce"]) / a.iters
        say(f"configs[4] {out['configs4_ms_per_iter']:.3f} ms per iteration")
    out["stats_end"] = collnet_stats()
    print("RESULT " + json.dumps(out), flush=True)
    # tear down under a deadline: the report is out, a teardown that blocks
    # (RCCL's proxy threads) must not hold the run
    import threading
    threading.Timer(30.0, lambda: os._exit(3)).start()
    dist.destroy_process_group()
    os._exit(0)


def launch(world: int, same_gpu: bool, numel: int = 1 << 22, iters: int = 5, channels: int = 0,
           algo: str | None = None, log_dir: str | None = None, timeout: float = 600,
           port: int | None = None, extra_env: dict | None = None, switch_topo: bool = False,
           allow_collnet: bool = False) -> dict:
    """Run `world` ranks (child processes) and gather their reports.
    allow_collnet: offer the CollNet table to RCCL (SWITCHML_COLLNET_RCCL=1)
    with NCCL_ALGO=CollNetDirect and the switch node — the experiment that
    hangs on RCCL 7.2 (give it a short timeout)."""
    if allow_collnet:
        algo = algo or "CollNetDirect"
        switch_topo = True
        extra_env = dict(extra_env or {}, SWITCHML_COLLNET_RCCL="1")
    session = uuid.uuid4().hex[:10]
    if log_dir:
        os.makedirs(log_dir, exist_ok=True)
    import tempfile
    out_dir = log_dir or tempfile.mkdtemp(prefix="sml_rccl_collnet_")
    # rendezvous through a FileStore in a fresh directory unless a port is
    # asked for (a port picked here and bound by rank 0 later can be taken
    # in between)
    store_dir = tempfile.mkdtemp(prefix="sml_rccl_pg_")
    rdzv = ["--port", str(port)] if port else ["--init", os.path.join(store_dir, "store")]
    procs, files = [], []
    for r in range(world):
        env = worker_env(os.environ, r, world, 0 if same_gpu else r, session, channels, algo, log_dir, extra_env)
        cmd = [sys.executable, "-u", "-m", "switchml_amd.rccl_collnet", "--rank", str(r), "--world", str(world),
               "--device", str(0 if same_gpu else r), "--numel", str(numel),
               "--iters", str(iters), "--topo-dir", out_dir] + rdzv
        if switch_topo:
            cmd.append("--switch-topo")
        f = open(os.path.join(out_dir, f"rank{r}.out"), "w+")
        files.append(f)
        procs.append(subprocess.Popen(cmd, env=env, stdout=f, stderr=subprocess.STDOUT, text=True))
    t0 = time.time()
    t_end = t0 + timeout
    last = t0
    while any(p.poll() is None for p in procs):
        if time.time() > t_end:
            for q in procs:
                q.kill()
            break
        if any(p.poll() not in (None, 0) for p in procs):
            time.sleep(5)   # one rank failed: give the others a moment, then stop them
            for q in procs:
                if q.poll() is None:
                    q.kill()
            break
        if time.time() - last > 10:
            last = time.time()
            tail = []
            for f in files:
                f.flush()
                with open(f.name, errors="replace") as g:
                    ls = [l for l in g.read().splitlines() if l.startswith("[rank")]
                tail.append(ls[-1] if ls else "-")
            print(f"[rccl_collnet] {time.time() - t0:.0f} s: " + " | ".join(tail), file=sys.stderr, flush=True)
        time.sleep(0.2)
    for p in procs:
        p.wait()
    import shutil
    shutil.rmtree(store_dir, ignore_errors=True)
    outs = []
    for f in files:
        with open(f.name, errors="replace") as g:
            outs.append(g.read())
        f.close()
    ranks, tails = [], []
    for o in outs:
        res = [l for l in o.splitlines() if l.startswith("RESULT ")]
        ranks.append(json.loads(res[-1][7:]) if res else None)
        tails.append(o.strip().splitlines()[-12:])
    rep = {"world": world, "same_gpu": same_gpu, "numel": numel, "channels": channels, "algo": algo,
           "extra_env": extra_env or {}, "switch_topo": switch_topo,
           "returncodes": [p.returncode for p in procs], "ranks": ranks}
    if any(r is None for r in ranks) or any(p.returncode for p in procs):
        rep["tails"] = tails
    ok = all(r is not None for r in ranks) and all(p.returncode == 0 for p in procs)
    rep["allow_collnet"] = allow_collnet
    rep["iallreduce_calls"] = [r["stats_end"]["iallreduce"] if r else None for r in ranks]
    rep["collnet_dispatched_by_rccl"] = bool(ok and all(
        r["stats_after_first"]["iallreduce"] > r["stats_before"]["iallreduce"] for r in ranks))
    rep["collnet_declined"] = bool(ok and all(r["stats_end"].get("declined", 0) >= 1 for r in ranks))
    rep["hand_int_exact"] = bool(ok and all(r.get("hand_int_exact", False) for r in ranks))
    rep["ok"] = bool(ok and all(r["int_exact"] and r["hand_int_exact"] and r["int_equal_direct"] and r["normal_within_bound"]
                                for r in ranks)
                     and (rep["collnet_dispatched_by_rccl"] if allow_collnet else rep["collnet_declined"]))
    return rep


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--port", type=int, default=29655)
    ap.add_argument("--init", default="", help="(rank) FileStore path for the rendezvous (instead of --port)")
    ap.add_argument("--numel", type=int, default=1 << 22)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--same-gpu", action="store_true")
    ap.add_argument("--channels", type=int, default=0, help="NCCL_MAX_NCHANNELS (0 = RCCL's default)")
    ap.add_argument("--algo", default="", help="NCCL_ALGO for the ranks ('' = RCCL's tuner)")
    ap.add_argument("--allow-collnet", action="store_true",
                    help="offer the CollNet table to RCCL (SWITCHML_COLLNET_RCCL=1, CollNetDirect, switch node)")
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE for the ranks (repeatable)")
    ap.add_argument("--switch-topo", action="store_true",
                    help="add a switch node to each worker's RCCL topology (CollNetDirect's precondition)")
    ap.add_argument("--topo-dir", help="(rank) where the topology files go")
    ap.add_argument("--log-dir")
    ap.add_argument("--out")
    ap.add_argument("--timeout", type=float, default=600.0, help="seconds before the ranks are killed")
    a = ap.parse_args(argv)
    if a.rank is not None:
        rank_main(a)
        return 0
    rep = launch(a.world, a.same_gpu, a.numel, a.iters, a.channels, a.algo or None, a.log_dir,
                 extra_env=dict(kv.split("=", 1) for kv in a.env), switch_topo=a.switch_topo,
                 timeout=a.timeout, allow_collnet=a.allow_collnet)
    if a.log_dir:
        lines = []
        for f in sorted(os.listdir(a.log_dir)):
            with open(os.path.join(a.log_dir, f), errors="replace") as fh:
                lines += [f"{f}: {l.rstrip()}" for l in fh
                          if any(k in l for k in ("SWITCHML", "SwitchML", "CollNet", "collnet", "Collnet", "NET/",
                                                  "Plugin", "WARN", "Algo", "nNodes", "nodes"))]
        rep["rccl_log"] = lines[:200]
    s = json.dumps(rep, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)
    print(s)
    return 0 if rep["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
