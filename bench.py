"""Routing-table build benchmark (BASELINE.json metric: APSP pairs/sec +
routing-table build wall-clock, 16k-node graph at 1/2/4/8 MI355X).

One "step" = one full routing build of the 16,384-node complete undirected
graph (config C3: latency U{1..300} ms, loss U[0,0.01], self-loops, seed 3):
from the CSR resident in HBM to the n x n (latency, loss) table resident in
HBM (all-gathered on every rank for N > 1).  value = n^2 pairs / step time.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--nodes 16384]
Multi-GPU: launched by torch.distributed.run, one rank per GPU (RCCL).
Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X constants (/opt/skills/guides/MI355X_MICROARCH.md): 256 CUs x 4 SIMD-32,
# one wave64 VALU op per 2 cycles per SIMD -> 128 int32 lane-ops/clk/CU at 2.4 GHz.
VALU_LANE_OPS_PEAK = 256 * 128 * 2.4e9  # 78.6e12 int32 lane-ops/s
# FP64 VALU ops (v_add_f64, v_min_f64) issue at half that rate (spec: FP64 vector
# 78.6 TF vs FP32 157.3 TF; tools/valu_bench measured 36.5e12 lane-ops/s).  One
# lexicographic (latency, loss) relaxation on the f64-encoded path key is one
# v_add_f64 + one v_min_f64.
F64_LANE_OPS_PEAK = VALU_LANE_OPS_PEAK / 2  # 39.3e12
OPS_PER_RELAX = 2
RELAX_PEAK = F64_LANE_OPS_PEAK / OPS_PER_RELAX  # 19.66e12 relaxations/s


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--nodes", type=int, default=16384)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--cpu-baseline", dest="cpu_baseline", action="store_true", default=True)
    ap.add_argument("--no-cpu-baseline", dest="cpu_baseline", action="store_false")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-sources", type=int, default=0, help="0 = auto (~10-30 s of CPU work)")
    return ap.parse_args()


def cpu_baseline(n, seed, threads, sources):
    """The oracle's faithful restatement of compute_shortest_paths (hash-map
    Dijkstra per source + rayon-style pool), timed on a bounded sample of
    sources of the same graph; pairs/s extrapolated linearly (sources are
    independent, mod.rs:190-208)."""
    from oracle import oracle as O
    from shadow_amd import synth

    src, dst, lat, loss = synth.complete_graph(n, seed)
    g = O.Graph(False, np.arange(n), src, dst, lat, loss)
    nodes = np.arange(n, dtype=np.uint32)
    if sources <= 0:
        # calibrate: one source per thread, then scale to ~15 s
        t0 = time.perf_counter()
        O.compute_shortest_paths(g, nodes, threads=threads, mode=0, src_count=threads)
        dt = time.perf_counter() - t0
        sources = int(max(threads, min(n, threads * max(1, int(15.0 / max(dt, 1e-3))))))
    t0 = time.perf_counter()
    O.compute_shortest_paths(g, nodes, threads=threads, mode=0, src_count=sources)
    dt = time.perf_counter() - t0
    return {"value": sources * n / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"{sources} of {n} sources of the same C3 graph, faithful hash-map Dijkstra "
                      f"(oracle mode 0), {dt:.1f} s wall, extrapolated linearly to pairs/s"}


def measured_traffic(n, kernel_tag="phase 3 rest"):
    """HBM bytes per launch of the dominant kernel from the latest committed
    PMC summary (profiles/rNN_pmc_traffic.json, FETCH_SIZE + WRITE_SIZE passes
    of rocprofv3 on this same config), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    for f in reversed(files):
        d = json.load(open(f))
        if str(n) not in d.get("config", ""):
            continue
        for k, v in d.get("kernels", {}).items():
            if kernel_tag in k:
                return v["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


def main():
    args = parse_args()
    import torch
    import torch.distributed as dist

    from shadow_amd import NetworkGraph, synth
    from shadow_amd.plan import RoutingPlan

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n_gpus = max(args.gpus, world)
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = local_rank

    n = args.nodes
    row_ptr, col, lat, loss = synth.complete_csr(n, args.seed)
    g = NetworkGraph(n, np.arange(n, dtype=np.uint32), row_ptr, col, lat, loss, directed=False)
    nodes = np.arange(n, dtype=np.uint32)
    plan = RoutingPlan(g, nodes, device=dev)
    del row_ptr, col, lat, loss, g
    if world > 1:
        from shadow_amd import dist as sdist
        sdist.bind(plan, rank, world, local_rank, transport=os.environ.get("SRT_COMM", "rccl"))

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        plan.run()
    barrier()
    step_ms = []
    p3_ms, p3_launches, p3_work = 0.0, 0, 0.0
    t_all0 = time.perf_counter()
    for _ in range(args.steps):
        t0 = time.perf_counter()
        plan.run()
        step_ms.append((time.perf_counter() - t0) * 1e3)
        a, b, w, _ = plan.kernel_stats()
        p3_ms += a
        p3_launches += b
        p3_work += w
    barrier()
    elapsed = time.perf_counter() - t_all0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{dev}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    plan.fetch(table=False)  # connectivity check + min latency (not timed)

    if rank == 0:
        ms_per_step = elapsed * 1e3 / args.steps
        pairs = n * n
        value = pairs / (elapsed / args.steps)
        # dominant kernel: FW phase-3 "rest" launches; work = tiles x B^3 relaxations;
        # its algorithmic HBM traffic = every tile read + written once (B^2 keys of
        # 8 B each way per B^3 relaxations; the panels are L2/MALL-resident)
        relax_per_launch = p3_work / max(p3_launches, 1)
        B_TILE = 128
        avg_launch_s = (p3_ms / 1e3) / max(p3_launches, 1)
        achieved = relax_per_launch / avg_launch_s
        traffic, traffic_src = measured_traffic(n)
        roofline = {"bound": "valu", "achieved": achieved / 1e12, "peak": RELAX_PEAK / 1e12, "unit": "Trelax/s",
                    "frac": achieved / RELAX_PEAK, "traffic": traffic, "traffic_unit": "HBM bytes per launch",
                    "traffic_source": traffic_src,
                    "algorithmic_hbm_bytes_per_launch": relax_per_launch / B_TILE * 2 * 8 if B_TILE else None,
                    "kernel": "minplus_tile_kernel<double, 0> (FW phase 3, rest)", "avg_launch_ms": avg_launch_s * 1e3,
                    "relax_per_launch": relax_per_launch,
                    "peak_basis": f"{F64_LANE_OPS_PEAK / 1e12:.1f}e12 f64 VALU lane-ops/s / {OPS_PER_RELAX} ops "
                                  f"(v_add_f64 + v_min_f64) per relaxation"}
        cpu = None
        if args.cpu_baseline and world == 1:
            cpu = cpu_baseline(n, args.seed, args.cpu_threads, args.cpu_sources)
        out = {
            "metric": "APSP pairs/sec (routing-table build, 16k-node graph)",
            "value": value, "unit": "pairs/s", "n_gpus": n_gpus, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64" if "f64key" in plan.describe() else "u64", "data": "synthetic (seeded complete graph, latency U{1..300} ms, loss U[0,0.01])",
            "config": {"workload": f"C3: {n}-node complete undirected GML graph, use_shortest_path=true, "
                                   f"blocked Floyd-Warshall", "nodes": n, "pairs": pairs,
                       "parallelism": f"rows{n_gpus}" if n_gpus > 1 else "single",
                       "plan": plan.describe(), "step_ms": [round(x, 3) for x in step_ms],
                       "build_wallclock_ms": ms_per_step},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    plan.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
