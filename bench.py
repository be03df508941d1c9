"""Routing-table build benchmark (BASELINE.json metric: APSP pairs/sec +
routing-table build wall-clock, 16k-node graph at 1/2/4/8 MI355X).

Default workload (--config c3): one "step" = one full routing build of the
16,384-node complete undirected graph (config C3: latency U{1..300} ms, loss
U[0,0.01], self-loops, seed 3), from the CSR resident in HBM to the n x n
(latency, loss) table resident in HBM (all-gathered on every rank for N > 1):
the latency closure plus the exact-loss pass.  value = n^2 pairs / step time.
Beside it the line carries the end-to-end build through the C ABI
(srt_compute_shortest_paths: host CSR in, srt_path[n*n] in the caller's host
buffer out, every validation and PCIe copy included) -- BASELINE.md's t_build.

Other configs (same JSON shape):
  --config c1   1,000-node complete graph through its GML TEXT: parse + build +
                fetch to the host per step; the reference CPU path (faithful
                restatement, all sources) is timed in full beside it
  --config c2   4,096-node complete graph (blocked Floyd-Warshall, 1 GPU)
  --config c2nc the C2 graph with 30% of its edges dropped (dense, not complete:
                key width from the eccentricity proof)
  --config c4   100,000-node Barabasi-Albert graph, m=4 (batched sparse sweep)
  --config c5   1M packets/round send_packet decision on the C1 table (packets/s)

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
Multi-GPU: one rank per GPU (RCCL), launched by torch.distributed.run; run as
`python bench.py --gpus N` without a launcher it starts the N ranks itself
(before any GPU call) and exits with their status.  Prints one JSON line on
rank 0.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X constants (/opt/skills/guides/MI355X_MICROARCH.md; profiles/r01_valu_bench.txt)
VALU_LANE_OPS_PEAK = 256 * 64 * 2.4e9  # 39.3e12 lane-ops/s (one 4-cycle VALU slot per lane per cycle)
# u16 latency keys: v_pk_add_u16 + v_pk_min_u16 relax 2 keys = 1 slot per relaxation;
# u32: 2 v_add_u32 (double rate) + 1 v_min3_u32 per 2 relaxations = 1 slot (an
# optimistic basis: the mix measures 28.1 Trelax/s, tools/valu_bench.hip)
RELAX_PEAK = {"f16": VALU_LANE_OPS_PEAK / 0.75, "u16": VALU_LANE_OPS_PEAK / 1.0, "u32": VALU_LANE_OPS_PEAK / 1.0, "f64": VALU_LANE_OPS_PEAK / 2.0,
              "u64": VALU_LANE_OPS_PEAK / 4.0}
RELAX_BASIS = {"f16": "2 v_pk_add_f16 + 1 v_pk_minimum3_f16 per 4 relaxations (2 keys per VGPR, two k-steps "
                      "folded by the 3-input min) = 0.75 VALU slot",
               "u16": "v_pk_add_u16 + v_pk_min_u16 per 2 relaxations (2 keys per VGPR) = 1 VALU slot",
               "u32": "2 v_add_u32 (issued at twice the rate) + 1 v_min3_u32 per 2 relaxations = 1 VALU slot",
               "f64": "v_add_f64 + v_min_f64 = 2 VALU slots", "u64": "v_lshl_add_u64 + v_cmp + 2 v_cndmask = 4 slots"}
HBM_PEAK = 8.0e12  # B/s
MALL_GATHER_PEAK = 8.6e12  # B/s: random rows of a 38 MB table, Infinity Cache (MI355X_MICROARCH.md)

CONFIGS = {
    "c1": dict(kind="gml", nodes=1000, seed=1),
    "c2": dict(kind="complete", nodes=4096, seed=2),
    # C2 with 30% of its undirected edges dropped: dense but not complete, so
    # the key width comes from the eccentricity proof (fw_ecc_bound), not the
    # longest edge
    "c2nc": dict(kind="dense", nodes=4096, seed=2, drop=0.3),
    "c3": dict(kind="complete", nodes=16384, seed=3),
    # C3 with ns-resolution latencies (a sub-ms offset on every edge): g = 1 ns,
    # so the closure runs u32 keys and the loss pass the scan fold
    "c3ns": dict(kind="complete", nodes=16384, seed=3, ns=True),
    "c4": dict(kind="ba", nodes=100_000, seed=4, m=4),
    "c5": dict(kind="packets", nodes=1000, seed=5, hosts=10_000, packets=1_000_000),
}
PATH_DTYPE = np.dtype([("lat", "<u8"), ("loss", "<f4"), ("pad", "<u4")])


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--nodes", type=int, default=0, help="override the config's node count")
    ap.add_argument("--in-use", dest="in_use", type=int, default=0,
                    help="c4: number of in-use nodes (default: all)")
    ap.add_argument("--seed", type=int, default=-1)
    ap.add_argument("--cpu-baseline", dest="cpu_baseline", action="store_true", default=True)
    ap.add_argument("--no-cpu-baseline", dest="cpu_baseline", action="store_false")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the CPUs this process may use")
    ap.add_argument("--cpu-sources", type=int, default=0, help="0 = auto (~10-30 s of CPU work)")
    ap.add_argument("--no-e2e", dest="e2e", action="store_false", default=True)
    ap.add_argument("--no-cold", dest="cold", action="store_false", default=True,
                    help="skip the cold first-call legs (fresh processes) of the dense configs")
    ap.add_argument("--cold-child", dest="cold_child", default="", choices=["", "plain", "init"],
                    help=argparse.SUPPRESS)
    ap.add_argument("--exchange", default="auto", choices=["auto", "none", "allgather"],
                    help="N > 1: 'allgather' (the default, 'auto') = the communicator-bound build the north_star "
                         "names: rows all-gathered over RCCL so every rank holds the whole table (the line's value; "
                         "the no-exchange share is measured after it and carried as config.no_exchange); 'none' = "
                         "LEVEL / SSSP rows sharded with no collective as the value (each rank's rows stay in its HBM)")
    ap.add_argument("--tbuild-child", dest="tbuild_child", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--algo", default="auto", choices=["auto", "fw", "sssp", "level"],
                    help="kernel family (default: AUTO, the library's priced choice -- what the drop-in runs)")
    ap.add_argument("--rank-share", dest="rank_share", type=int, default=0,
                    help="measurement only: one GPU builds rank 0's rows of an N-rank row-sharded build "
                         "(srt_plan_shard_rows(N, 0): exactly that rank's work, no exchange exists) and prints "
                         "its time; not a bench line")
    ap.add_argument("--emulate-ranks", dest="emulate_ranks", type=int, default=0,
                    help="measurement only (dense FW, 1 GPU): time one rank of an N-rank run -- 1/N of the "
                         "block-rows plus the pivot owner's chain every round, no collectives; the table "
                         "is not valid and no bench line is printed, only the timing")
    return ap.parse_args()


def cpu_share():
    """Threads the CPU baseline runs on: the CPUs this process may use (rayon's
    default pool is every logical CPU it sees), capped by the job's CPU share
    when the box declares one (OMP_NUM_THREADS), plus the CPU model."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(aff, share) if share > 0 else aff
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return threads, aff, model


def cpu_baseline(og, nodes, threads, sources, label, target_s=15.0, mode=0, full=False):
    """The oracle's faithful restatement of compute_shortest_paths (mode 0:
    hash-map Dijkstra per source, the `nodes.contains` filter, per-source map,
    merged map; rayon-style pool) -- or its array-based variant (mode 1, the
    same algorithm without the hash maps: an "opt-cpu" for honesty) -- timed on
    a bounded sample of sources of the same graph (all of them when full);
    pairs/s extrapolated linearly (sources are independent, mod.rs:190-208)."""
    from oracle import oracle as O

    n = len(nodes)
    if full:
        sources = n
    elif sources <= 0:
        # calibrate: one source per thread, then scale to ~target_s
        t0 = time.perf_counter()
        O.compute_shortest_paths(og, nodes, threads=threads, mode=mode, src_count=threads)
        dt = time.perf_counter() - t0
        sources = int(max(threads, min(n, threads * max(1, int(target_s / max(dt, 1e-3))))))
    t0 = time.perf_counter()
    O.compute_shortest_paths(og, nodes, threads=threads, mode=mode, src_count=sources)
    dt = time.perf_counter() - t0
    what = ("faithful hash-map Dijkstra (oracle mode 0)" if mode == 0 else
            "array-score Dijkstra, same algorithm without the hash maps (oracle mode 1)")
    _, aff, model = cpu_share()
    return {"value": sources * n / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "cpu_model": model, "cpus_visible": aff,
            # BASELINE.md 4 asks for every logical CPU (rayon's default pool) and
            # 256 sampled sources; the bench contract bounds the sample to ~10-30 s
            # and a GPU-box job may use its CPU share only (OMP_NUM_THREADS), so
            # the all-CPU figure is a linear projection, stated as one
            "threads_note": (f"{threads} threads = this job's CPU share of the {aff} visible CPUs "
                             f"(OMP_NUM_THREADS on the GPU box); sources are independent (mod.rs:190-208)"),
            "projected_all_cpus": {"value": sources * n / dt * aff / max(threads, 1), "cores": aff,
                                   "how": "linear projection from the measured threads, not measured"},
            "sample": (f"all {n} sources" if sources == n else f"{sources} of {n} sources") +
                      f" of the same {label} graph, {what}, {dt:.2f} s wall" +
                      ("" if sources == n else ", extrapolated linearly to pairs/s"),
            **({} if sources >= min(256, n) else {
                "why_not_256": (f"BASELINE.md 4's 256-source sample would take ~{dt * 256 / sources:.0f} s on "
                                f"{threads} threads; the bench contract bounds the CPU leg to ~10-30 s, so "
                                f"{sources} sources (the per-source cost is flat: sources are independent)")})}


def measured_traffic(args, kernel_tag, schedule):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC
    summary (profiles/rNN*_pmc_traffic.json: FETCH_SIZE and WRITE_SIZE passes of
    rocprofv3 on this same workload and schedule, gfx950 corrections applied),
    or None.  A summary counts only if its config name, node count and recorded
    schedule (key type, rounds per launch, ranks) match this run's."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    for f in reversed(files):
        d = json.load(open(f))
        cfg = d.get("config", "")
        if not cfg.startswith(args.config.upper() + " ") or (args.nodes and str(args.nodes) not in cfg):
            continue
        if d.get("schedule") != schedule:
            continue
        # several instantiations may carry the tag (the level family's probe
        # launches use a smaller variant): the dominant one moved the most bytes
        hits = [v for k, v in d.get("kernels", {}).items() if kernel_tag in k]
        if hits:
            v = max(hits, key=lambda v: v["hbm_bytes_per_launch"] * v.get("dispatches", 1))
            return v["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


def packet_traffic():
    """HBM bytes of one C5 round's kernels (round_kernel + pack/stats; r05 and
    before: draw_kernel + decide_kernel) from the newest committed C5 PMC
    summary of the current kernel, or None."""
    import glob
    for f in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))):
        d = json.load(open(f))
        if not d.get("config", "").startswith("C5 "):
            continue
        ks = d.get("kernels", {})
        if not any(k.startswith("round_kernel") for k in ks):  # an older kernel shape (draw + decide)
            continue
        tot = sum(v["hbm_bytes_per_launch"] for k, v in ks.items() if k.startswith(("round_kernel", "stats_kernel")))
        if tot:
            return tot, os.path.relpath(f, ROOT)
    return None, None


def frontier_traffic(args, schedule, launches):
    """HBM bytes per launch of the frontier path: every fr_* kernel's bytes per
    dispatch x its dispatches, over the run's launches, from the newest committed
    PMC summary of this workload and schedule (see measured_traffic)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    for f in reversed(files):
        d = json.load(open(f))
        cfg = d.get("config", "")
        if not cfg.startswith(args.config.upper() + " ") or d.get("schedule") != schedule:
            continue
        tot = sum(v["hbm_bytes_per_launch"] * v["dispatches"] for k, v in d.get("kernels", {}).items()
                  if k.startswith("fr_") and not k.startswith("fr_emit"))
        if tot:
            return tot / max(d.get("launches", launches), 1), os.path.relpath(f, ROOT)
    return None, None


class Dist:
    def __init__(self):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        # rehearsal of the N-rank schedule on a one-GPU box (SRT_BENCH_ONE_DEVICE=1:
        # every rank on cuda:0, barrier / max over gloo); never the measured setup
        self.one_device = os.environ.get("SRT_BENCH_ONE_DEVICE") == "1"
        self.dev = 0 if self.one_device else self.local_rank
        if self.world > 1:
            torch.cuda.set_device(self.dev)
            if self.one_device:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local_rank))

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()
        self.torch.cuda.synchronize(self.dev)

    def max_over_ranks(self, x):
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device="cpu" if self.one_device else f"cuda:{self.dev}")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def timed_builds(plan, D, steps, warmup):
    for _ in range(warmup):
        plan.run()
    D.barrier()
    step_ms = []
    k_ms, k_launches, k_work, k_tiles = 0.0, 0, 0.0, 0
    t_all0 = time.perf_counter()
    for _ in range(steps):
        t0 = time.perf_counter()
        plan.run()
        step_ms.append((time.perf_counter() - t0) * 1e3)
        a, b, w, _ = plan.kernel_stats()
        k_tiles += plan.kernel_tiles()
        k_ms += a
        k_launches += b
        k_work += w
    D.barrier()
    elapsed = D.max_over_ranks(time.perf_counter() - t_all0)
    return elapsed, step_ms, k_ms, k_launches, k_work, k_tiles


ALGOS = {"auto": 0, "fw": 1, "sssp": 2, "level": 3}


def e2e_build(g, nodes, reps=3, algo=0):
    """BASELINE.md t_build: srt_compute_shortest_paths from the host CSR to the
    srt_path table in the caller's (pre-touched, reused) host buffer -- plan
    creation and validation, the CSR upload, the build, the download -- as the
    Rust shim would call it.  Best of `reps` calls."""
    from shadow_amd import _lib

    L = _lib.lib()
    n = len(nodes)
    out = np.empty(n * n, PATH_DTYPE)  # the caller's table: pages touched once, like a reused Vec
    out.view(np.uint8).fill(0)
    nodes = np.ascontiguousarray(nodes, np.uint32)
    csr = g.csr()
    opts = _lib.SrtOpts(algo, -1, 0, 0)
    best, times = None, []
    for _ in range(reps):
        err, mn = _lib.SrtErr(), C.c_uint64()
        t0 = time.perf_counter()
        rc = L.srt_compute_shortest_paths(C.byref(csr), nodes.ctypes.data_as(C.POINTER(C.c_uint32)), n,
                                          out.ctypes.data_as(C.POINTER(_lib.SrtPath)), C.byref(mn), C.byref(opts),
                                          C.byref(err))
        dt = time.perf_counter() - t0
        _lib.check(rc, err)
        best = dt if best is None else min(best, dt)
        times.append(round(dt * 1e3, 2))
    return {"ms": best * 1e3, "pairs_per_s": n * n / best, "calls": reps, "call_ms": times,
            "first_call_note": "the process's first call also pins the 192 MB download staging (behind its closure) "
                               "and cannot use the piece-pipelined upload, which needs that staging",
            "span": "srt_compute_shortest_paths: host CSR (borrowed) -> srt_path[n*n] in the caller's host buffer; "
                    "validation, CSR upload, build, table download and plan teardown included"}


def routing_info_builds(g, nodes, reps=3, algo=0):
    """generate_routing_info as Shadow calls it (sim_config.rs:424-461):
    srt_routing_info_build from the host CSR to the RoutingInfo (the table kept
    in its downloaded record form, decoded per path()).  Best of `reps`."""
    from shadow_amd import RoutingInfo
    times = []
    rb = 0
    for _ in range(reps):
        t0 = time.perf_counter()
        ri = RoutingInfo.build(g, nodes, algo=algo)
        times.append((time.perf_counter() - t0) * 1e3)
        rb = ri.record_bytes()
        ri.close()
    return {"ms": min(times), "call_ms": [round(x, 2) for x in times], "record_bytes": rb,
            "span": "srt_routing_info_build: host CSR -> RoutingInfo (validation, upload, build, download of the "
                    "table's records, plan teardown)"}


def cold_child(args):
    """One fresh process, one first call (the bench's --cold-child mode): 'init'
    calls srt_init_async first thing -- Shadow would, before its config and GML
    parsing -- and the graph is built meanwhile; 'plain' does not, so the call
    pays the HIP runtime start, the kernels' code-object loads and the pinning
    of the transfer staging."""
    t_start = time.perf_counter()
    import shadow_amd
    if args.cold_child == "init":
        shadow_amd.init_async(0)
    from shadow_amd import NetworkGraph, RoutingInfo, synth
    cfg = CONFIGS[args.config]
    n = args.nodes or cfg["nodes"]
    seed = cfg["seed"] if args.seed < 0 else args.seed
    if cfg["kind"] == "dense":
        row_ptr, col, lat, loss = synth.dense_csr(n, synth.dense_graph(n, seed, drop=cfg["drop"]))
    else:
        row_ptr, col, lat, loss = synth.complete_csr(n, seed, edges=synth.complete_graph_ns(n, seed)
                                                     if cfg.get("ns") else None)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    t1 = time.perf_counter()
    ri = RoutingInfo.build(g, nodes)
    t2 = time.perf_counter()
    print(json.dumps({"mode": args.cold_child, "first_call_ms": (t2 - t1) * 1e3,
                      "graph_build_s": t1 - t_start, "record_bytes": ri.record_bytes(),
                      "smallest_latency_ns": ri.get_smallest_latency_ns()}), flush=True)
    ri.close()


def cold_calls(args):
    """The cold first call in fresh processes, without and with srt_init_async."""
    out = {}
    for mode in ("plain", "init"):
        cmd = [sys.executable, os.path.abspath(__file__), "--cold-child", mode, "--config", args.config]
        if args.nodes:
            cmd += ["--nodes", str(args.nodes)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode != 0 or not line:
            raise SystemExit(f"cold child ({mode}) failed: {r.stderr[-2000:]}")
        out[mode] = json.loads(line[-1])
    return {"plain_first_call_ms": out["plain"]["first_call_ms"], "init_first_call_ms": out["init"]["first_call_ms"],
            "graph_build_s": out["init"]["graph_build_s"], "record_bytes": out["init"]["record_bytes"],
            "what": "srt_routing_info_build as the first GPU call of a fresh process: 'plain' pays HIP start-up, "
                    "code-object loads and the pinning of the transfer staging; 'init' called srt_init_async "
                    "at process start, overlapped with building the graph (Shadow: config + GML parsing)"}


def synth_graph(args, cfg):
    """The config's dense graph as a NetworkGraph (complete / dense kinds)."""
    from shadow_amd import NetworkGraph, synth
    n = args.nodes or cfg["nodes"]
    seed = cfg["seed"] if args.seed < 0 else args.seed
    if cfg["kind"] == "dense":
        row_ptr, col, lat, loss = synth.dense_csr(n, synth.dense_graph(n, seed, drop=cfg["drop"]))
    else:
        row_ptr, col, lat, loss = synth.complete_csr(n, seed, edges=synth.complete_graph_ns(n, seed)
                                                     if cfg.get("ns") else None)
    return NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)


def tbuild_child(args):
    """BASELINE.md's t_build at N GPUs as Shadow calls it: ONE process
    (generate_routing_info runs once, in Shadow's main thread,
    sim_config.rs:136-140) building with srt_opts.n_gpus = N -- one library
    thread and one plan per device, each device solving its share of the rows
    and downloading them over its own link.  Run by rank 0 of an N-rank bench
    as a child process after every rank released its plans."""
    from shadow_amd import RoutingInfo
    cfg = CONFIGS[args.config]
    g = synth_graph(args, cfg)
    n = g.n_nodes
    nodes = np.arange(n, dtype=np.uint32)
    same = os.environ.get("SRT_BENCH_ONE_DEVICE") == "1"
    N = args.tbuild_child
    out = {"n_gpus": N, "same_device": same}
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        ri = RoutingInfo.build(g, nodes, n_gpus=N, same_device=same, device=0)
        times.append((time.perf_counter() - t0) * 1e3)
        ri.close()
    out["routing_info_ms"] = min(times)
    out["routing_info_call_ms"] = [round(x, 2) for x in times]
    out["routing_info_pairs_per_s"] = n * n / (min(times) / 1e3)
    out["span"] = ("srt_routing_info_build with srt_opts.n_gpus = N from one process: host CSR -> RoutingInfo "
                   "(validation, upload, class CSRs, every device's rows solved and downloaded over its own link)")
    print(json.dumps(out), flush=True)


def tbuild_leg(args, N):
    """Rank 0: tbuild_child in a fresh process; its JSON, or the failure."""
    cmd = [sys.executable, os.path.abspath(__file__), "--tbuild-child", str(N), "--config", args.config]
    if args.nodes:
        cmd += ["--nodes", str(args.nodes)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    except subprocess.TimeoutExpired:
        return {"error": "t_build child timed out (600 s)"}
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not line:
        return {"error": f"t_build child failed (rc {r.returncode}): {(r.stderr or r.stdout)[-600:]}"}
    return json.loads(line[-1])


def gml_graph(n_nodes, seed):
    from shadow_amd import synth
    src, dst, lat, loss = synth.complete_graph(n_nodes, seed)
    return synth.gml_text(n_nodes, src, dst, lat, loss)


def bench_gml(args, cfg, D):
    """C1: a step = NetworkGraph::parse of the GML text (srt_gml_parse) + the
    routing build + the table in host memory (srt_compute_shortest_paths) --
    the reference's generate_routing_info span on this input.  The CPU
    reference path (oracle GML parse + faithful Dijkstra over all sources) is
    timed in full beside it."""
    from shadow_amd import NetworkGraph

    n_nodes = args.nodes or cfg["nodes"]
    seed = cfg["seed"] if args.seed < 0 else args.seed
    text = gml_graph(n_nodes, seed)
    nodes = np.arange(n_nodes, dtype=np.uint32)

    def step():
        g = NetworkGraph.parse(text)
        return e2e_build(g, nodes, reps=1)

    for _ in range(args.warmup):
        step()
    D.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    D.barrier()
    elapsed = D.max_over_ranks(time.perf_counter() - t0)
    out = None
    if D.rank == 0:
        per = elapsed / args.steps
        cpu = None
        if args.cpu_baseline:
            from oracle import oracle as O
            threads = args.cpu_threads or cpu_share()[0]
            t1 = time.perf_counter()
            og = O.gml_parse(text)
            parse_s = time.perf_counter() - t1
            cpu = cpu_baseline(og, nodes, threads, 0, "C1", full=True)
            cpu["sample"] += f"; plus the oracle's GML parse ({parse_s:.2f} s, not in value)"
        # the closure's key type, from a plan over the same graph (not timed)
        from shadow_amd.plan import RoutingPlan
        probe = RoutingPlan(NetworkGraph.parse(text), nodes, device=D.dev)
        desc = probe.describe()
        probe.close()
        out = {
            "metric": "APSP pairs/sec (routing-table build from GML text, 1k-node graph)",
            "value": D.world * n_nodes * n_nodes / per, "unit": "pairs/s", "n_gpus": D.world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": per * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": desc.split(":")[1][:3] if desc.startswith("fw") else "u64",
            "data": "synthetic (seeded complete GML graph, latency U{1..300} ms, loss U[0,0.01])",
            "config": {"workload": f"C1: {n_nodes}-node complete undirected GML graph, use_shortest_path=true: "
                                   f"GML text -> srt_gml_parse -> srt_compute_shortest_paths -> host table",
                       "nodes": n_nodes, "pairs": n_nodes * n_nodes, "gml_bytes": len(text), "plan": desc,
                       "parallelism": "replicas" if D.world > 1 else "single"},
            "roofline": None,
            "cpu_baseline": cpu,
        }
    return out


def bench_graph(args, cfg, D):
    from shadow_amd import NetworkGraph, synth
    from shadow_amd.plan import RoutingPlan

    n_nodes = args.nodes or cfg["nodes"]
    seed = cfg["seed"] if args.seed < 0 else args.seed
    if cfg["kind"] == "complete":
        edges = synth.complete_graph_ns(n_nodes, seed) if cfg.get("ns") else None
        row_ptr, col, lat, loss = synth.complete_csr(n_nodes, seed, edges=edges)
        g = NetworkGraph(n_nodes, np.arange(n_nodes, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
        nodes = np.arange(n_nodes, dtype=np.uint32)
        if cfg.get("ns"):
            label = (f"{args.config.upper()}: {n_nodes}-node complete undirected graph, latencies in ns (the C3 "
                     f"ms values plus a seeded sub-ms offset: g = 1 ns), CSR built directly")
            data = "synthetic (seeded complete graph, latency U{1..300} ms + U{0..999999} ns, loss U[0,0.01])"
        else:
            label = (f"{args.config.upper()}: {n_nodes}-node complete undirected graph (CSR built directly; the "
                     f"same values as the GML text of synth.gml_text, GML ingest not in this step)")
            data = "synthetic (seeded complete graph, latency U{1..300} ms, loss U[0,0.01])"
        og_args = edges
        del row_ptr, col, lat, loss
    elif cfg["kind"] == "dense":
        edges = synth.dense_graph(n_nodes, seed, drop=cfg["drop"])
        row_ptr, col, lat, loss = synth.dense_csr(n_nodes, edges)
        g = NetworkGraph(n_nodes, np.arange(n_nodes, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
        nodes = np.arange(n_nodes, dtype=np.uint32)
        label = (f"{args.config.upper()}: {n_nodes}-node dense undirected graph (the complete graph of seed "
                 f"{seed} with {cfg['drop']:.0%} of its edges dropped, self-loops kept)")
        data = f"synthetic (seeded dense graph, latency U{{1..300}} ms, loss U[0,0.01], {cfg['drop']:.0%} edges dropped)"
        og_args = edges
        del row_ptr, col, lat, loss
    else:
        src, dst, lat, loss = synth.barabasi_albert(n_nodes, cfg["m"], seed)
        g = NetworkGraph.from_edges(n_nodes, src, dst, lat, loss, directed=False)
        n = args.in_use or n_nodes
        nodes = (np.arange(n_nodes, dtype=np.uint32) if n == n_nodes else
                 np.sort(np.random.default_rng(seed).choice(n_nodes, n, replace=False)).astype(np.uint32))
        label = (f"{args.config.upper()}: {n_nodes}-node Barabasi-Albert graph (m={cfg['m']}, avg degree "
                 f"{2 * len(src) / n_nodes:.1f} incl. self-loops), {len(nodes)} in use")
        data = "synthetic (seeded BA graph, latency U{1..300} ms, loss U[0,0.01])"
        og_args = (src, dst, lat, loss)
    if args.emulate_ranks > 1:
        os.environ["SRT_FW_EMULATE_RANKS"] = str(args.emulate_ranks)
    plan = RoutingPlan(g, nodes, algo=ALGOS[args.algo], device=D.dev)
    ranks = 1
    transport = None
    if args.rank_share > 1 and D.world == 1:
        # rank 0's share of an N-rank build whose class CSR is sharded too: its
        # slice built, the all-gather of the slices modelled as a wait (25 us +
        # received bytes / 300 GB/s; SRT_LVL_SHARD_EMU=0 builds the whole CSR)
        os.environ.setdefault("SRT_LVL_SHARD_EMU", "1")
        plan.shard_rows(args.rank_share, 0)
        elapsed, step_ms, k_ms, k_launches, k_work, _ = timed_builds(plan, D, args.steps, args.warmup)
        t = plan.timing()
        ms = elapsed * 1e3 / args.steps
        print(json.dumps({"rank_share": {"ranks": args.rank_share, "rank": 0, "config": args.config,
                                         "plan": plan.describe(), "ms_per_step": ms,
                                         "solve_ms_per_step": k_ms / args.steps,
                                         "device_total_ms_last": t["total_ms"],
                                         "implied_value_pairs_per_s": len(nodes) ** 2 / (ms / 1e3),
                                         "csr_shard_emulated": os.environ.get("SRT_LVL_SHARD_EMU") == "1",
                                         "note": "rank 0's rows of an N-rank row-sharded build, measured alone on one "
                                                 "GPU: its slice of the class CSR, the slices' all-gather modelled as a "
                                                 "wait (25 us + received bytes / 300 GB/s), its rows solved (the table "
                                                 "rows are not exchanged); the implied value assumes the N ranks run "
                                                 "concurrently on N GPUs"}}),
              flush=True)
        plan.close()
        return None
    exchange = args.exchange if args.exchange != "auto" else ("allgather" if D.world > 1 else "none")
    if D.world > 1 and exchange == "none" and plan.describe().startswith(("level", "sssp")):
        # independent source rows (mod.rs:190-208): each rank builds its share
        # of the rows into its own HBM, no collective in the data path -- the
        # table stays distributed by rows, as the in-process build downloads it
        plan.shard_rows(D.world, D.rank)
    elif D.world > 1:
        from shadow_amd import dist as sdist
        # the collectives' transport is part of the measurement: native RCCL on
        # the plan's streams unless SRT_COMM names another; a failure to set it
        # up ends the run (no silent fallback to a different transport)
        transport = os.environ.get("SRT_COMM", "torch" if D.one_device else "rccl")
        sdist.bind(plan, D.rank, D.world, D.dev, transport=transport)
    desc = plan.describe()
    if " ranks=" in desc:
        ranks = int(desc.split(" ranks=")[1].split()[0])
    elif " shard=" in desc:
        ranks = int(desc.split(" shard=")[1].split("/")[1].split()[0])
    if ranks != D.world:
        raise SystemExit(f"plan bound to {ranks} ranks but WORLD_SIZE={D.world}")
    elapsed, step_ms, k_ms, k_launches, k_work, k_tiles = timed_builds(plan, D, args.steps, args.warmup)
    if args.emulate_ranks > 1:
        t = plan.timing()
        print(json.dumps({"emulated_ranks": args.emulate_ranks, "config": args.config, "ms_per_step":
                          elapsed * 1e3 / args.steps, "rest_ms_per_step": k_ms / args.steps,
                          "rest_launches_per_step": k_launches // args.steps,
                          "tail_ms_last": t["loss_ms"], "build_ms_last": t["total_ms"],
                          "note": "rank 0 of an N-rank run on one GPU: closure schedule on the closed D, loss pass "
                                  "on its own rows; collectives modelled as waits (25 us + bytes / 300 GB/s)"}),
              flush=True)
        plan.close()
        return None
    timing = plan.timing()  # phase breakdown of the last timed build
    desc = plan.describe()  # after the runs: the first one adds what it measured (e.g. sym=triangle)
    plan.fetch(table=False)  # connectivity check + min latency (not timed)
    plan.close()
    n = len(nodes)
    no_exchange = None
    if D.world > 1 and transport is not None and desc.startswith(("level", "sssp")):
        # the same build with rows sharded and no collective (each rank's rows
        # stay in its HBM): what the exchange costs, carried beside the value
        p2 = RoutingPlan(g, nodes, algo=ALGOS[args.algo], device=D.dev)
        p2.shard_rows(D.world, D.rank)
        e2, st2, _, _, _, _ = timed_builds(p2, D, args.steps, args.warmup)
        p2.close()
        no_exchange = {"ms_per_step": e2 * 1e3 / args.steps, "value": n * n / (e2 / args.steps),
                       "step_ms": [round(x, 3) for x in st2],
                       "what": "rows sharded with no collective (srt_plan_shard_rows): each rank's rows stay in its "
                               "HBM, no rank holds the table -- the exchange-free share of the build, not the value"}
    t_build = None
    if D.world > 1 and args.e2e and cfg["kind"] in ("complete", "dense"):
        D.barrier()  # every rank's plans are released: the devices are free for one process
        if D.rank == 0:
            t_build = tbuild_leg(args, D.world)
        D.barrier()
    e2e = None
    if args.e2e and D.world == 1 and cfg["kind"] in ("complete", "dense"):
        e2e = e2e_build(g, nodes, algo=ALGOS[args.algo])
        e2e["routing_info"] = routing_info_builds(g, nodes, algo=ALGOS[args.algo])
        if args.cold:
            e2e["cold"] = cold_calls(args)
    out = None
    if D.rank == 0:
        pairs = n * n
        ms_per_step = elapsed * 1e3 / args.steps
        avg_launch_s = (k_ms / 1e3) / max(k_launches, 1)
        work_per_launch = k_work / max(k_launches, 1)
        key = desc.split(":")[1][:3] if desc.startswith(("fw", "level")) else "u64"
        if desc.startswith("level"):
            # level solve: the launches write the table (12 B a pair: u64 latency
            # + f32 loss) and walk the pruned class CSRs (L2/MALL resident)
            # algorithmic bytes: the 12-byte table pair written, and every class
            # entry a row walks (8 B; the class CSRs exceed the L2, the PMC
            # summary shows them fetched from beyond it)
            visits_run = timing["edge_visits"]  # the last timed build's rows, counted by the kernel
            visits_launch = visits_run / max(k_launches // max(args.steps, 1), 1)
            alg_bytes = work_per_launch * 12 + visits_launch * 8
            achieved = alg_bytes / avg_launch_s
            visits = visits_run // max(n, 1)
            lmax = int(desc.split(" lmax=")[1].split("(")[0])
            sh = int(desc.split(" q=")[1].split()[0]) if " q=" in desc else 0  # quantized: bucket width
            schedule = {"family": "level", "lmax": lmax, "rows_per_launch": int(work_per_launch // max(n, 1))}
            if sh:
                schedule["q"] = sh
            kname = "level_q_kernel" if sh else "level_solve_kernel"
            traffic, traffic_src = measured_traffic(args, kname, schedule)
            roofline = {
                "bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": achieved / HBM_PEAK, "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE: gfx950 16-B/lane correction)",
                "traffic_source": (f"{traffic_src}: committed rocprofv3 PMC summary of this workload and schedule, "
                                   f"not measured in this run" if traffic_src else
                                   "no committed PMC summary for this workload/schedule"),
                "schedule": schedule,
                "kernel": (f"{kname} (per-source bucket Dijkstra over the class CSRs, one workgroup a row"
                           + (f"; buckets of {sh} units, u64 (latency, loss) keys)" if sh else ")")),
                "avg_launch_ms": avg_launch_s * 1e3, "pairs_per_launch": work_per_launch,
                "algorithmic_bytes_per_launch": alg_bytes,
                "basis": "12 B per table pair written (u64 latency + f32 loss) + 8 B per class-CSR entry the rows "
                         "walk (counted by the kernel; the class CSRs exceed the 4 MB L2 of an XCD)",
                "edge_visits_per_row": visits,
                "edge_visits_per_s": visits_launch / avg_launch_s,
                # the class entries are gathered from beyond L2 (Infinity Cache): the guide's measured
                # random-row rate from a table of that size is the second ceiling; the table write alone
                # is the floor every build pays
                "second_peak": {"what": "Infinity Cache random-row gather (MI355X_MICROARCH.md 'Indexed rows: "
                                        "gather into LDS', 38 MB table: 8.6 TB/s chip-wide; C3's class CSR is 43 MB)",
                                "peak": MALL_GATHER_PEAK / 1e9, "unit": "GB/s", "frac": achieved / MALL_GATHER_PEAK},
                "write_floor": {"bytes_per_launch": work_per_launch * 12,
                                "frac_of_hbm": work_per_launch * 12 / avg_launch_s / HBM_PEAK,
                                "what": "the 12-B table pairs alone over the launch time"}}
            algo = (f"level solve: per-source bucket (Dial) Dijkstra over the edges <= {lmax} units (a bound proved "
                    f"by probe rows), loss folded in the same pass"
                    + (f"; quantized buckets of {sh} units (the shortest edge)" if sh else ""))
        elif desc.startswith("fw"):
            B_TILE = 128
            kbytes = {"f16": 2, "u16": 2, "u32": 4}.get(key, 8)
            achieved = work_per_launch / avg_launch_s
            rounds = k_work / max(k_tiles * B_TILE ** 3, 1)
            schedule = {"key": key, "launch_rounds": int(round(rounds)), "ranks": D.world,
                        "tiles": "triangle" if "sym=triangle" in desc else "square"}
            traffic, traffic_src = measured_traffic(args, "(phase 3 rest)", schedule)
            peak = RELAX_PEAK[key]
            roofline = {
                "bound": "valu", "achieved": achieved / 1e12, "peak": peak / 1e12, "unit": "Trelax/s",
                "frac": achieved / peak, "traffic": traffic,
                # f16 keys: also on the 1-slot-per-relaxation basis of the u16 kernel
                "frac_1slot_basis": achieved / VALU_LANE_OPS_PEAK,
                "traffic_unit": "HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE: gfx950 16-B/lane correction)",
                "traffic_source": (f"{traffic_src}: committed rocprofv3 PMC summary of this workload and schedule, "
                                   f"not measured in this run" if traffic_src else
                                   "no committed PMC summary for this workload/schedule"),
                "schedule": schedule,
                # every C tile read + written once per launch (A/B panels hit L2/MALL);
                # triangle launches also write each off-diagonal tile's mirror
                "algorithmic_hbm_bytes_per_launch": k_tiles / max(k_launches, 1) * B_TILE * B_TILE * kbytes *
                                                    (3 if "sym=triangle" in desc else 2),
                "rounds_per_tile": rounds,
                "kernel": (f"minplus_u16_kernel<0, SYM, F16={key == 'f16'}>" if key in ("f16", "u16") else
                           f"minplus_{key if key == 'u32' else 'glds'}_kernel<0>") + " (FW phase 3, rest)",
                "avg_launch_ms": avg_launch_s * 1e3, "relax_per_launch": work_per_launch,
                "peak_basis": f"{VALU_LANE_OPS_PEAK / 1e12:.1f}e12 VALU lane-op slots/s; {key} keys: "
                              f"{RELAX_BASIS[key]} per relaxation (f64 keys would peak at 19.7, the SURVEY's "
                              f"5-int32-op u64 basis at 7.86 Trelax/s)"}
            algo = f"blocked Floyd-Warshall ({key} latency closure) + exact-loss fold over the tight DAG"
        else:
            achieved = work_per_launch / avg_launch_s
            launches_per_step = k_launches // max(args.steps, 1)
            sweeps_per_launch = timing["sparse_sweeps"] / max(launches_per_step, 1)
            frontier = desc.startswith("sssp:frontier")
            if frontier:
                schedule = {"state": "frontier-u16", "blocks": int(desc.split(" blocks=")[1].split()[0]),
                            "first": int(desc.split(" first=")[1].split()[0]) if " first=" in desc else 0,
                            "seed": desc.split(" seed=")[1].split()[0],
                            "source_order": desc.split(" order=")[1].split()[0]}
                traffic, traffic_src = frontier_traffic(args, schedule, launches_per_step)
                kernel = ("fr_lat_sweep_kernel + fr_tight_kernel + fr_loss_sweep_kernel: every sweep of one launch "
                          "(its blocks of 512 sources)")
                algo = "latency-first frontier sweeps (u16 latencies, then f32 loss over the tight DAG)"
            else:
                state = desc.split("state=")[1].split()[0] if "state=" in desc else "keys"
                schedule = {"state": state,
                            "words_per_lane": int(desc.split(" R=")[1].split()[0]) if " R=" in desc else 0,
                            "source_order": desc.split(" order=")[1].split()[0]}
                per_sweep, traffic_src = measured_traffic(args, "(sssp_sweep)", schedule)
                traffic = per_sweep * sweeps_per_launch if per_sweep else None
                kernel = "sssp_sweep_kernel (all sweeps of one launch)"
                algo = "batched sparse sweep"
            roofline = {
                "bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": achieved / HBM_PEAK,
                "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (PMC bytes of the launch's kernels, per launch)",
                "traffic_source": (f"{traffic_src}: committed rocprofv3 PMC summary of this workload and layout, "
                                   f"not measured in this run" if traffic_src else
                                   "no committed PMC summary for this workload/layout"),
                "schedule": schedule,
                "kernel": kernel,
                "avg_launch_ms": avg_launch_s * 1e3, "launches_per_step": launches_per_step,
                "sweeps_per_launch": sweeps_per_launch,
                "algorithmic_bytes_per_launch": work_per_launch,
                "basis": "12 B x (E_in + V) per source (SURVEY.md 8(d)), E_in = in-edges without self-loops"}
        cpu = cpu_opt = None
        if args.cpu_baseline and D.world == 1:
            from oracle import oracle as O
            threads = args.cpu_threads or cpu_share()[0]
            if og_args is None:  # complete graph: regenerate the edge list (the CSR was built directly)
                og = O.Graph(False, np.arange(n_nodes), *synth.complete_graph(n_nodes, seed))
            else:
                og = O.Graph(False, np.arange(n_nodes), *og_args)
            cpu = cpu_baseline(og, nodes, threads, args.cpu_sources, args.config.upper())
            cpu_opt = cpu_baseline(og, nodes, threads, args.cpu_sources, args.config.upper(), target_s=8.0,
                                   mode=1)
        out = {
            "metric": f"APSP pairs/sec (routing-table build, {n_nodes // 1000 if n_nodes >= 1000 else n_nodes}"
                      f"{'k' if n_nodes >= 1000 else ''}-node graph)",
            "value": pairs / (elapsed / args.steps), "unit": "pairs/s", "n_gpus": ranks, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": key,
            "data": data,
            "config": {"workload": f"{label}, use_shortest_path=true, {algo}", "nodes": n_nodes, "in_use": n,
                       "pairs": pairs,
                       "parallelism": ("single" if ranks == 1 else
                                       f"rows{ranks} (no exchange: each rank's rows stay in its HBM)"
                                       if " shard=" in desc else f"rows{ranks} (all-gathered over {transport})"),
                       "transport": transport, "nranks": ranks,
                       "plan": desc, "step_ms": [round(x, 3) for x in step_ms], "build_wallclock_ms": ms_per_step,
                       "create_device_ms": timing["create_device_ms"],
                       "fresh_graph": {"ms": ms_per_step + timing["create_device_ms"],
                                       "value": pairs / ((ms_per_step + timing["create_device_ms"]) / 1e3),
                                       "what": "a build of a graph seen for the first time: the step plus the device "
                                               "work of plan creation (bound proofs, level probes, symmetry check) -- "
                                               "Shadow builds once per process (sim_config.rs:136-140)"},
                       "no_exchange": no_exchange, "t_build": t_build,
                       "phases_last_build": {"device_total_ms": timing["total_ms"],
                                             "dominant_ms": timing["dominant_ms"],
                                             "exact_loss_pass_ms": timing["loss_ms"],
                                             "tight_edges": timing["tight_edges"],
                                             "loss_fold": "level" if timing["loss_fold"] else "scan"},
                       "e2e": e2e},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "cpu_baseline_opt": cpu_opt,
        }
    return out


def bench_packets(args, cfg, D):
    """C5: one round = srt_packet_batch over 1M packets (10k hosts on the C1
    nodes, loss U[0,0.25]), inputs resident in HBM; value = packets/s.
    Replicas only: each rank runs its own round (per-host RNG streams shard by
    source host, no exchange)."""
    import torch

    from oracle import oracle as O
    from shadow_amd import NetworkGraph, synth
    from shadow_amd.plan import RoutingPlan

    n_nodes, hosts, n_pkts = cfg["nodes"], cfg["hosts"], cfg["packets"]
    seed = cfg["seed"] if args.seed < 0 else args.seed
    src, dst, lat, loss = synth.complete_graph(n_nodes, seed, loss_max=0.25)
    g = NetworkGraph.from_edges(n_nodes, src, dst, lat, loss)
    plan = RoutingPlan(g, np.arange(n_nodes, dtype=np.uint32), device=D.dev).run()
    r0, r1 = 1_000_000_000, 1_000_000_000 + 5 * synth.MS
    pk, host_ptr, _ = synth.packet_round(hosts, n_nodes, n_pkts, seed, r0, r1)
    rng0 = synth.host_rng_states(hosts, general_seed=1)
    dev = torch.device("cuda", D.dev)
    t_pk = torch.from_numpy(pk.view(np.uint8).copy()).to(dev)
    t_hp = torch.from_numpy(host_ptr.view(np.int32).copy()).to(dev)
    t_rng = torch.from_numpy(rng0.view(np.int64).copy()).to(dev)
    t_f = torch.zeros(n_pkts, dtype=torch.int32, device=dev)
    t_d = torch.zeros(n_pkts, dtype=torch.int64, device=dev)
    t_c = torch.zeros(n_nodes * n_nodes, dtype=torch.int64, device=dev)
    t_s = torch.full((2,), -1, dtype=torch.int64, device=dev)
    stream = torch.cuda.ExternalStream(plan.stream_ptr(), device=dev)

    # diagnostics only (never a reported line): SRT_BENCH_NO_COUNTERS drops the per-pair counters
    t_cc = None if os.environ.get("SRT_BENCH_NO_COUNTERS") else t_c

    def one():
        plan.packet_batch(t_pk, t_hp, t_rng, r1, 0, 2**62, t_f, t_d, t_cc, t_s, sync=False)

    for _ in range(args.warmup):
        one()
    plan.sync()
    D.barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        one()
    ev1.record(stream)
    plan.sync()
    D.barrier()
    elapsed = D.max_over_ranks(time.perf_counter() - t0)
    dev_ms = ev0.elapsed_time(ev1) / args.steps
    # the round's event push (srt_packet_events, worker.rs:629-639), timed
    # after the headline loop on the last round's flags: reported beside the
    # decision rate, not folded into it
    dst_host = ((pk["dst_row"].astype(np.int64) + n_nodes * (np.arange(n_pkts) % max(1, hosts // n_nodes)))
                % hosts).astype(np.int32)
    t_dh = torch.from_numpy(dst_host).to(dev)
    t_base = torch.zeros(hosts, dtype=torch.int64, device=dev)
    t_eid = torch.zeros(n_pkts, dtype=torch.int64, device=dev)
    t_ord = torch.zeros(n_pkts, dtype=torch.int32, device=dev)
    t_ptr = torch.zeros(hosts + 1, dtype=torch.int32, device=dev)
    ev_reps = max(3, args.steps)
    plan.packet_events(t_hp, t_f, t_d, t_dh, hosts, t_base, t_eid, t_ord, t_ptr)
    ee0, ee1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    te0 = time.perf_counter()
    ee0.record(stream)
    for _ in range(ev_reps):  # asynchronous calls, one status check at the end
        plan.packet_events(t_hp, t_f, t_d, t_dh, hosts, t_base, t_eid, t_ord, t_ptr, check=False)
    ee1.record(stream)
    plan.packet_events_status()
    events_ms = (time.perf_counter() - te0) * 1e3 / ev_reps
    events_dev_ms = ee0.elapsed_time(ee1) / ev_reps
    out = None
    if D.rank == 0:
        per_round = elapsed / args.steps
        bytes_per_round = n_pkts * 52 + hosts * 64
        traffic, traffic_src = packet_traffic()
        cpu = None
        if args.cpu_baseline and D.world == 1:
            table = plan.fetch()
            rng = rng0.copy()
            t0 = time.perf_counter()
            reps = 0
            while time.perf_counter() - t0 < 10.0:
                O.packet_batch(table.latency_ns, table.packet_loss, pk.view(O.PKT_DTYPE), rng, r1, 0, 2**62)
                reps += 1
            dt = time.perf_counter() - t0
            _, aff, model = cpu_share()
            cpu = {"value": reps * n_pkts / dt, "unit": "packets/s", "cores": 1, "kind": "port",
                   "cpu_model": model, "cpus_visible": aff,
                   "sample": f"{reps} rounds of the same 1M-packet batch through the oracle's sequential "
                             f"send_packet restatement (one thread: Shadow decides a host's packets on the one "
                             f"worker thread that runs the host), {dt:.1f} s"}
        out = {
            "metric": "batched send_packet decisions/sec (1M packets/round)", "value": D.world * n_pkts / per_round,
            "unit": "packets/s", "n_gpus": D.world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": per_round * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u64", "data": "synthetic (seeded packet round, 10k hosts on the C1 nodes, loss U[0,0.25])",
            "config": {"workload": "C5: 1M packets/round, latency lookup + per-host xoshiro256++ loss drops",
                       "packets": n_pkts, "hosts": hosts, "parallelism": "replicas"},
            "roofline": {"bound": "hbm", "achieved": bytes_per_round / (dev_ms / 1e3) / 1e9,
                         "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": bytes_per_round / (dev_ms / 1e3) / HBM_PEAK, "traffic": traffic,
                         "traffic_unit": "HBM bytes per round (FETCH_SIZE + WRITE_SIZE of round_kernel + stats_kernel)",
                         "traffic_source": (f"{traffic_src}: committed rocprofv3 PMC summary of this workload, not "
                                            f"measured in this run" if traffic_src else
                                            "no committed PMC summary for this workload"),
                         "kernel": "round_kernel + stats_kernel (one round: per-host draws in LDS, decisions)",
                         "device_ms_per_round": dev_ms,
                         "basis": "52 B/packet + 64 B/host (SURVEY.md 8(d))"},
            "cpu_baseline": cpu,
            "events": {"ms_per_round": events_ms, "device_ms_per_round": events_dev_ms,
                       "sent": int(t_ptr[-1].item()),
                       "what": "srt_packet_events on the round's sent packets: per-host event ids, stable sort by "
                               "destination, deliver times sorted within each destination (the queue pop order); "
                               "asynchronous calls, wall clock per round with one status check at the end, and the "
                               "device time of the same calls"},
        }
    plan.close()
    return out


def spawn_ranks(args):
    """--gpus N > 1 without a launcher: start the N ranks under
    torch.distributed.run as child processes (this process has not touched the
    GPU) and exit with their status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    args = parse_args()
    if args.cold_child:
        cold_child(args)
        return
    if args.tbuild_child:
        tbuild_child(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world == 1:
        sys.exit(spawn_ranks(args))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    cfg = CONFIGS[args.config]
    D = Dist()
    if cfg["kind"] == "packets":
        out = bench_packets(args, cfg, D)
    elif cfg["kind"] == "gml":
        out = bench_gml(args, cfg, D)
    else:
        out = bench_graph(args, cfg, D)
    if out is not None:
        print(json.dumps(out), flush=True)
    D.close()


if __name__ == "__main__":
    main()
