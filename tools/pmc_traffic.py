#!/usr/bin/env python3
"""Turn a tools/gpu_profile.sh run into committed evidence under profiles/.

Reads gpurun_out/prof_<tag>/ (rocprofv3 kernel-trace stats + one PMC pass per
counter) and writes
  profiles/<tag>_kernel_stats.csv   -- rocprofv3 --stats summary, verbatim
  profiles/<tag>_pmc.json           -- per-kernel HBM bytes per launch
  profiles/traffic_<workload>.json  -- what bench.py reports as roofline.traffic

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports exactly half of a wide
(16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Both our kernels use only 16-B loads/stores.

    python tools/pmc_traffic.py <tag> <workload> [lost]

<workload> is a bench.py workload name or a custom "k,m,bs,S" shape; [lost]
(default 1) = lost data blocks per stripe of the profiled decode (bench.py
--lost), which scales the decode's algorithmic bytes.  traffic_<workload>.json
is written for named workloads only.
"""
from __future__ import annotations

import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "")


def build_id_of(info: str | None) -> str | None:
    """The "src:<id>" token of an xec_build_info() string (None if absent)."""
    for tok in (info or "").split():
        if tok.startswith("src:"):
            return tok[4:]
    return None


def git_head() -> str | None:
    import subprocess
    r = subprocess.run(["git", "-C", str(ROOT), "rev-parse", "--short=12", "HEAD"],
                       capture_output=True, text=True)
    return r.stdout.strip() or None


def per_kernel(csv_path: Path) -> dict[str, list[float]]:
    agg: dict[str, list[float]] = {}
    for r in csv.DictReader(open(csv_path)):
        agg.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return agg


def main():
    tag, workload = sys.argv[1], sys.argv[2]
    lost = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    src = ROOT / "gpurun_out" / f"prof_{tag}"
    dst = ROOT / "profiles"
    dst.mkdir(exist_ok=True)
    shutil.copy(src / "trace" / "kt_kernel_stats.csv", dst / f"{tag}_kernel_stats.csv")
    fetch = per_kernel(src / "pmc_FETCH_SIZE" / "pmc_counter_collection.csv")
    write = per_kernel(src / "pmc_WRITE_SIZE" / "pmc_counter_collection.csv")
    stats = {short(r["Name"]): r for r in csv.DictReader(open(src / "trace" / "kt_kernel_stats.csv"))}

    from bench import WORKLOADS, algorithmic_bytes, workload_shape
    k, m, bs, S, _ = workload_shape(workload)
    b_enc, b_dec = algorithmic_bytes(S, k, m, bs)
    algo = {"xec::encode_kernel": b_enc, "xec::decode_kernel": b_dec * lost,
            "xec::decode_class_kernel": b_dec * lost, "xec::decode_list_kernel": b_dec * lost,
            "xec::decode_arglist_kernel": b_dec * lost, "xec::decode_argmask_kernel": b_dec * lost,
            "xec::decode_devlist_kernel": b_dec * lost}

    kernels = {}
    for name in sorted(set(fetch) & set(write)):
        base = name.split("<")[0]
        if base not in algo:
            continue
        # only the default shape (one granule per lane); the PMC passes run
        # without the bench's legs (tools/gpu_profile.sh), so every launch
        # left is the headline batch
        targs = [a.strip() for a in name.split("<", 1)[1].rstrip(">").split(",")]
        if len(targs) > 1 and targs[1] != "1":
            continue
        f_kib = sum(fetch[name]) / len(fetch[name])
        w_kib = sum(write[name]) / len(write[name])
        hbm = int(round((2 * f_kib + w_kib) * 1024))
        st = stats.get(name, {})
        avg_ns = float(st["AverageNs"]) if st else None
        kernels[name] = {
            "launches_sampled": len(fetch[name]),
            "FETCH_SIZE_KiB": round(f_kib, 1), "WRITE_SIZE_KiB": round(w_kib, 1),
            "hbm_bytes_per_launch": hbm,
            "algorithmic_bytes_per_launch": algo[base],
            "traffic_over_algorithmic": round(hbm / algo[base], 4),
            "rocprof_avg_ns": avg_ns,
            "rocprof_calls": int(st["Calls"]) if st else None,
            "achieved_GBps_algorithmic": round(algo[base] / avg_ns, 1) if avg_ns else None,
        }
    info_f = src / "build_info.txt"
    build_info = info_f.read_text().strip() if info_f.exists() else None
    build_id = build_id_of(build_info)
    out = {"tag": tag, "build_info": build_info, "build_id": build_id,
           "git_head_at_collection": git_head(),
           "workload": workload, "k": k, "m": m, "block_bytes": bs, "stripes": S,
           "lost_per_stripe": lost,
           "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) KiB * 1024 (gfx950 FETCH_SIZE halves 16-B streams)",
           "kernels": kernels}
    (dst / f"{tag}_pmc.json").write_text(json.dumps(out, indent=1) + "\n")
    enc = [v for n, v in kernels.items() if n.startswith("xec::encode_kernel")]
    if enc and workload in WORKLOADS:
        traffic = {"source": f"profiles/{tag}_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE)",
                   # the library the profile measured (xec_build_info "src:<id>"): bench.py
                   # reports whether it is the library the line ran
                   "build_id": build_id,
                   # the same session's kernel trace: bench.py's roofline.achieved /
                   # frac are algorithmic bytes / its AverageNs (bench.rocprof_avg_ns)
                   "timing_source": f"profiles/{tag}_kernel_stats.csv",
                   "encode_hbm_bytes_per_launch": enc[0]["hbm_bytes_per_launch"],
                   "encode_algorithmic_bytes_per_launch": enc[0]["algorithmic_bytes_per_launch"]}
        dec = [v for n, v in kernels.items() if n.startswith("xec::decode")]
        if dec:
            traffic["decode_hbm_bytes_per_launch"] = dec[0]["hbm_bytes_per_launch"]
            traffic["decode_kernel"] = [n for n in kernels if n.startswith("xec::decode")][0]
        (dst / f"traffic_{workload}.json").write_text(json.dumps(traffic, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
