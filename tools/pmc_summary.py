#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/ (committed evidence).

traffic per launch of the dominant kernel =
  (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes
FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads 1/2 of the bytes of
wide (16 B/lane) coalesced reads (MI355X_MICROARCH.md §HBM), which is what the
row gathers are, so it is doubled; WRITE_SIZE is exact for 16-B/lane stores.
"""
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def counter(path, name, kernel_sub="train_"):
    vals = []
    for r in csv.DictReader(open(path)):
        if kernel_sub in r["Kernel_Name"] and r["Counter_Name"] == name:
            vals.append(float(r["Counter_Value"]))
    return vals


def main(tag, key):
    src = ROOT / "gpurun_out" / f"prof_{tag}"
    dst = ROOT / "profiles"
    dst.mkdir(exist_ok=True)
    shutil.copy(src / "kt" / "kt_kernel_stats.csv", dst / f"{tag}_kernel_stats.csv")
    fetch = counter(src / "fetch" / "fetch_counter_collection.csv", "FETCH_SIZE")
    write = counter(src / "write" / "write_counter_collection.csv", "WRITE_SIZE")
    stats = list(csv.DictReader(open(src / "kt" / "kt_kernel_stats.csv")))
    k = [r for r in stats if "train_" in r["Name"]][0]
    bench = json.loads((src / "kt_bench.json").read_text())
    key = key or bench["config"]["traffic_key"]
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    traffic = (2 * f_kib + w_kib) * 1024
    rec = {
        "tag": tag,
        "workload": bench["config"]["workload"],
        "kernel": k["Name"],
        "launches": int(k["Calls"]),
        "avg_duration_ms_rocprof": float(k["AverageNs"]) / 1e6,
        "avg_launch_ms_bench_events": bench["roofline"]["avg_launch_ms"],
        "algorithmic_bytes_per_launch": bench["roofline"]["algorithmic_bytes_per_launch"],
        "FETCH_SIZE_KiB_per_launch": f_kib,
        "WRITE_SIZE_KiB_per_launch": w_kib,
        "hbm_traffic_bytes_per_launch": traffic,
        "hbm_traffic_bytes_per_launch_uncorrected": (f_kib + w_kib) * 1024,
        "traffic_GBps": traffic / (float(k["AverageNs"]) * 1e-9) / 1e9,
    }
    (dst / f"{tag}_pmc.json").write_text(json.dumps(rec, indent=1) + "\n")
    rec["bench_ms_per_step_same_process"] = bench["ms_per_step"]
    (dst / f"{tag}_pmc.json").write_text(json.dumps(rec, indent=1) + "\n")
    tf = dst / "pmc_traffic.json"
    allrec = json.loads(tf.read_text()) if tf.exists() else {}
    allrec[key] = {"traffic": int(traffic), "source": f"profiles/{tag}_pmc.json",
                   "avg_duration_ms_rocprof": rec["avg_duration_ms_rocprof"]}
    tf.write_text(json.dumps(allrec, indent=1) + "\n")
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    # key: the profiled bench line's own config.traffic_key unless given
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
