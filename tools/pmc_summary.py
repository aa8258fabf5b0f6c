"""Turn one tools/gpu_profile.sh output directory into the committed profile summaries:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats (same command as bench.py)
  profiles/<tag>_bench.json         the bench line of that session
  profiles/<tag>_pmc.json           stepper FETCH_SIZE / WRITE_SIZE per launch and per event
  profiles/pmc_c3.json / pmc_c3_bins.json  the latest of the above for the row / bin store, read by
                                    bench.py for roofline.traffic and the hbm_requests / valu_issue views
  profiles/<tag>_pmc_calibration.json  bytes per access of the calibration kernels
Usage: python tools/pmc_summary.py gpurun_out/prof_<tag> <tag>
"""
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(src, tag):
    prof = os.path.join(REPO, "profiles")
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    bench = json.load(open(os.path.join(src, "bench.json")))
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(prof, f"{tag}_bench.json"))
    kstats = {r["Name"]: float(r["AverageNs"]) for r in rows(os.path.join(src, "kt", "kt_kernel_stats.csv"))}
    pmc = {}
    kname = "ssa_stepper_bins" if bench.get("store") == "bins" else "ssa_stepper"
    for counter, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write"), (None, "pmc_sq")):
        path = os.path.join(src, sub, "pmc_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in rows(path):
            if r["Kernel_Name"] in (kname, "ssa_hist"):
                d = pmc.setdefault(r["Kernel_Name"], {})
                if counter:
                    d[counter + "_bytes"] = float(r["Counter_Value"]) * 1024.0
                else:
                    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                d.update(VGPR_Count=int(r["VGPR_Count"]), SGPR_Count=int(r["SGPR_Count"]),
                         LDS_Block_Size=int(r["LDS_Block_Size"]), Grid_Size=int(r["Grid_Size"]))
    ev = bench["config"]["events_per_step"]
    st = pmc[kname]
    # which build the counters describe: bench.py reads the counter fields only while this digest matches
    # the kernel sources it runs (bench.kernel_sources_digest; gpu_profile.sh records it on the box)
    digest_path = os.path.join(src, "kernel_sources_sha256.txt")
    digest = open(digest_path).read().strip() if os.path.exists(digest_path) else None
    try:
        import subprocess

        head = subprocess.run(["git", "-C", REPO, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                              text=True).stdout.strip() or None
    except Exception:
        head = None
    out = {
        "round": tag,
        "git_head": head,
        "kernel_sources_sha256": digest,
        "workload": bench["config"]["workload"],
        "store": bench.get("store", "rows"),
        "kernel": kname,
        "events_per_launch": ev,
        "FETCH_SIZE_bytes_per_launch": st["FETCH_SIZE_bytes"],
        "WRITE_SIZE_bytes_per_launch": st["WRITE_SIZE_bytes"],
        "hbm_bytes_per_launch": st["FETCH_SIZE_bytes"] + st["WRITE_SIZE_bytes"],
        "read_bytes_per_event": st["FETCH_SIZE_bytes"] / ev,
        "write_bytes_per_event": st["WRITE_SIZE_bytes"] / ev,
        "read_requests_per_event": st["FETCH_SIZE_bytes"] / ev / 64.0,
        "write_requests_per_event": st["WRITE_SIZE_bytes"] / ev / 32.0,
        "stepper_avg_ns_rocprof": kstats.get(kname),
        "stepper_avg_ms_hip_events": bench["config"]["kernel_ms_avg"],
        "transactions_per_s": (st["FETCH_SIZE_bytes"] / 64.0 + st["WRITE_SIZE_bytes"] / 32.0)
        / (kstats[kname] * 1e-9),
        "correction": "none: the stepper makes no wide streaming reads (the gfx950 x2 FETCH_SIZE correction "
                      "applies to 16-B/lane coalesced reads, reproduced by the calibration stream_load_x4 "
                      "ratio 0.5); on this access shape one random 2-B load = one 64-B read request and one "
                      "random 2-B store = one 32-B write request (calibration file)",
        # the kernel instance the bench line timed (bench.py config.instance, ABI v7 ecdna_ssa_ctx_instance)
        "instance": bench["config"].get("instance"),
        "launch": {k: st[k] for k in ("VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Grid_Size")},
        "sq": {k: st[k] for k in st if k.startswith("SQ_")},
        "ssa_hist": pmc.get("ssa_hist"),
        "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of "
                  "`python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline` (tools/gpu_profile.sh)",
    }
    if "SQ_INSTS_VALU" in st:
        # SQ_INSTS_VALU counts wave instructions; one wave-event = 64 lane-events
        out["valu_insts_per_event"] = st["SQ_INSTS_VALU"] / ev
        out["valu_wave_insts_per_wave_event"] = st["SQ_INSTS_VALU"] / (ev / 64.0)
        out["salu_wave_insts_per_wave_event"] = st.get("SQ_INSTS_SALU", 0.0) / (ev / 64.0)
        out["lds_wave_insts_per_wave_event"] = st.get("SQ_INSTS_LDS", 0.0) / (ev / 64.0)
    json.dump(out, open(os.path.join(prof, f"{tag}_pmc.json"), "w"), indent=1)
    json.dump(out, open(os.path.join(prof, "pmc_c3_bins.json" if out["store"] == "bins" else "pmc_c3.json"), "w"),
              indent=1)
    cal = {}
    for counter, sub in (("FETCH_SIZE", "calib_fetch"), ("WRITE_SIZE", "calib_write")):
        p = os.path.join(src, sub, "pmc_counter_collection.csv")
        if os.path.exists(p):
            for r in rows(p):
                if not r["Kernel_Name"].startswith("__"):
                    cal.setdefault(r["Kernel_Name"], {})[counter + "_bytes"] = float(r["Counter_Value"]) * 1024
    if cal:
        acc = 67108864
        cj = {k: {c.replace("_bytes", "_bytes_per_access"): v / acc for c, v in d.items()}
              for k, d in cal.items() if k != "stream_load_x4"}
        if "stream_load_x4" in cal:
            cj["stream_load_x4"] = {"FETCH_SIZE_bytes": cal["stream_load_x4"]["FETCH_SIZE_bytes"],
                                    "true_bytes": 4 << 30,
                                    "ratio": cal["stream_load_x4"]["FETCH_SIZE_bytes"] / (4 << 30)}
        json.dump(cj, open(os.path.join(prof, f"{tag}_pmc_calibration.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
