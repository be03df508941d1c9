"""Condense one tools/profile_round.sh output directory into the files kept
under profiles/ (committed; gpurun_out/ is scratch):

  profiles/<tag>_bench.json          the bench JSON line
  profiles/<tag>_kernel_stats.csv    rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc_traffic.json    FETCH_SIZE / WRITE_SIZE per dispatch of
                                     every kernel (bench.py reads the dominant
                                     kernel's entry as roofline.traffic)

usage: python tools/summarize_profile.py gpurun_out/<tag> <tag> "<config text>" ['<schedule json>']
(the schedule -- key type, rounds per rest launch, ranks -- is what bench.py
matches before it quotes a summary's traffic for a run)
"""
import csv
import collections
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

LABELS = {
    "minplus_u16_kernel<0>": "phase 3 rest",
    "minplus_u16_kernel<0, 1>": "phase 3 rest",
    "minplus_u16_kernel<0, 3>": "phase 3 rest",
    "minplus_u16_kernel<0, 0, true>": "phase 3 rest",
    "minplus_u16_kernel<0, 1, true>": "phase 3 rest",
    "minplus_u16_kernel<0, 3, true>": "phase 3 rest",
    "minplus_u16_kernel<0, 0, false>": "phase 3 rest",
    "minplus_u16_kernel<0, 1, false>": "phase 3 rest",
    "minplus_u16_kernel<0, 3, false>": "phase 3 rest",
    "minplus_u16_kernel<5>": "phase 3 look-ahead (grouped)",
    "minplus_u32_kernel<0>": "phase 3 rest",
    "minplus_u32_kernel<5>": "phase 3 look-ahead (grouped)",
    "tight_loss_kernel": "exact-loss fold",
    "tight_flag_kernel": "tight-edge flags",
    "minplus_glds_kernel<double, 0>": "phase 3 rest",
    "minplus_glds_kernel<double, 4>": "phase 3 cross",
    "minplus_glds_kernel<double, 5>": "phase 3 cross (paired rounds)",
    "minplus_glds_kernel<double, 1>": "phase 2 row",
    "minplus_glds_kernel<double, 2>": "phase 2 col",
    "minplus_tile_kernel<double, 0>": "phase 3 rest",
    "sssp_sweep_kernel": "sssp_sweep",
    "fr_lat_sweep_kernel": "frontier latency sweep",
    "fr_tight_kernel": "frontier tight pass",
    "fr_loss_sweep_kernel": "frontier loss sweep",
    "fr_emit_kernel": "frontier emit",
    "decide_kernel": "packet decide",
    "level_solve_kernel": "level solve",
    "level_q_kernel": "quantized level solve",
    "edge_min_kernel": "shortest edge (quantized level probe)",
    "lvl_out_kernel": "level class CSR, out-rows",
    "lvl_in_kernel": "level class CSR, in-rows",
    "draw_kernel": "packet draw",
}


# FETCH_SIZE correction per kernel (MI355X_MICROARCH.md HBM section: x2 for
# 16-B/lane streaming reads, global_load and buffer_load ... lds alike).  The
# u16 / u32 tile kernels read C tiles and panels 16 B per lane; others as recorded
# (the f64 tile kernels' 8-B/lane C loads were calibrated 1:1 in r01).
FETCH_CORR = {"minplus_u32_kernel": 2.0, "minplus_u16_kernel": 2.0,
              # frontier sweeps: 128-B rows gathered 16 B a lane (8 lanes a line)
              "fr_lat_sweep_kernel": 2.0, "fr_tight_kernel": 2.0, "fr_loss_sweep_kernel": 2.0, "fr_emit_kernel": 2.0,
              # level solve: class entries gathered 16 B a lane (4 lanes a 64-B run)
              "level_solve_kernel": 2.0, "level_q_kernel": 2.0}


def short(name):
    n = name
    for pre in ("(anonymous namespace)::", "void ", "srt::"):
        n = n.replace(pre, "")
    return n.split("(")[0].strip()


def pmc(path, counter):
    """Counter KB summed per kernel and launch grid: one instantiation may run
    at several grids (the level family's create-time probes launch the build's
    solve kernel over a few sources), and the build's launches are the ones a
    bench line quotes.  The largest grid keeps the kernel's name; the others
    are keyed '<name> [grid N]'."""
    per = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = (short(r["Kernel_Name"]), int(r.get("Grid_Size") or 0))
            per[k] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    top = collections.defaultdict(int)
    for (k, g) in per:
        top[k] = max(top[k], g)
    return {(k if g == top[k] else f"{k} [grid {g}]"): (v, len(disp[(k, g)])) for (k, g), v in per.items()}


def main():
    src, tag, config = sys.argv[1], sys.argv[2], sys.argv[3]
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    bench = open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1]
    json.loads(bench)
    open(os.path.join(out, f"{tag}_bench.json"), "w").write(bench + "\n")
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(out, f"{tag}_kernel_stats.csv"))
    fetch, write = pmc(os.path.join(src, "pmc_fetch"), "FETCH_SIZE"), pmc(os.path.join(src, "pmc_write"), "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        fkb, fn = fetch.get(k, (0.0, 1))
        wkb, wn = write.get(k, (0.0, 1))
        label = next((v for p, v in LABELS.items() if k.startswith(p)), None)
        key = f"{k} ({label})" if label else k
        corr = next((v for p, v in FETCH_CORR.items() if k.startswith(p)), 1.0)
        kernels[key] = {"dispatches": max(fn, wn), "FETCH_SIZE_KB_per_launch": fkb / max(fn, 1),
                        "WRITE_SIZE_KB_per_launch": wkb / max(wn, 1), "fetch_correction": corr,
                        "hbm_bytes_per_launch": 1024.0 * (corr * fkb / max(fn, 1) + wkb / max(wn, 1))}
    # the PMC passes run one step without warmup: the frontier's launches of one step
    launches = (json.loads(bench).get("roofline") or {}).get("launches_per_step")
    doc = {"round": tag, "config": config, "launches": launches,
           "schedule": json.loads(sys.argv[4]) if len(sys.argv) > 4 else None,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (MI355X_MICROARCH.md "
                     "HBM section), KB per dispatch averaged over the dispatches of each kernel and launch grid (the "
                     "largest grid under the kernel's name, others as '[grid N]'). "
                     "hbm_bytes_per_launch = fetch_correction x FETCH_SIZE + WRITE_SIZE: x2 for the u32 tile "
                     "kernel (16-B/lane C-tile and LDS-DMA panel reads, the guide's gfx950 correction); 1 "
                     "elsewhere (raw counter: the f64 tile kernels' 8-B/lane C loads calibrated 1:1 in r01, "
                     "other widths uncalibrated).",
           "kernels": kernels}
    json.dump(doc, open(os.path.join(out, f"{tag}_pmc_traffic.json"), "w"), indent=1)
    print(json.dumps({k: round(v["hbm_bytes_per_launch"] / 1e6, 2) for k, v in kernels.items()}, indent=1))
    sq_dir = os.path.join(src, "pmc_sq")
    if os.path.isdir(sq_dir):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for f in glob.glob(os.path.join(sq_dir, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = (short(r["Kernel_Name"]), int(r.get("Grid_Size") or 0))
                per[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
        top = collections.defaultdict(int)
        for (k, g) in per:
            top[k] = max(top[k], g)
        per = {(k if g == top[k] else f"{k} [grid {g}]"): v for (k, g), v in per.items()}
        disp = {(k if g == top[k] else f"{k} [grid {g}]"): v for (k, g), v in disp.items()}
        sq = {}
        for k, c in per.items():
            n = max(len(disp[k]), 1)
            avg = {name: v / n for name, v in c.items()}
            wave = avg.get("SQ_WAVE_CYCLES", 0.0)
            row = {"per_dispatch": avg}
            if wave:
                row["frac_of_wave_cycles"] = {name: avg[name] / wave for name in
                                              ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                                               "SQ_ACTIVE_INST_VALU") if name in avg}
            sq[k] = row
        json.dump({"round": tag, "config": config,
                   "method": "one rocprofv3 --pmc pass (8 SQ counters + GRBM_GUI_ACTIVE), --steps 1; SQ cycle "
                             "counters are quad-cycles summed over waves, GRBM_GUI_ACTIVE summed over the 8 XCDs "
                             "(MI355X_MICROARCH.md)", "kernels": sq},
                  open(os.path.join(out, f"{tag}_pmc_sq.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
