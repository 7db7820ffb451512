#!/usr/bin/env python3
"""bench.py -- device-resident XOR-EC encode + single-erasure decode on MI355X.

One *step* = one encode pass over one batch + one single-erasure decode pass
over one batch (the reference's timed pair, src/benchmark/abstract_runner.hpp:
104-112), each through the C ABI of libxec_hip.so (include/xec.h).

Workload (BASELINE.json configs[2], the config the metric is quoted on):
k=16 data + m=1 parity, 1 MiB shards, 256 stripes per GPU (4 GiB data,
256 MiB parity), one lost data block per stripe, (7c) mod k.  Inputs are
resident in HBM before timing starts.  Three buffer sets rotate so that no
kernel reads bytes the kernel before it just wrote (the 256 MiB Infinity
Cache could serve them): step s encodes set s%3 and decodes set (s+2)%3, so
the decode of a set and the encode that wrote its parity (and the encode of a
set and the decode that rewrote its lost blocks) are always two kernels --
8+ GiB of traffic -- apart.

Multi-GPU: one process per GPU.  `python bench.py --gpus N` starts its own N
rank processes (launch_ranks: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set per
child, MASTER_ADDR 127.0.0.1) before anything touches the GPU; under
torch.distributed.run (WORLD_SIZE already set) it is one of the ranks.  Each
rank owns a contiguous stripe range (xec.partition.stripe_range) -- no
collective on the data path; barrier + max-over-ranks timing; value = all
ranks' bytes / max time ("weak").  RCCL ("nccl") carries the barrier, the
timing reductions and the config-5 scatter/gather leg.

    python bench.py [--gpus N] [--steps K] [--warmup W]

`--rehearse-cpu --dist-backend gloo` swaps the device calls for CPU stand-ins
(tools/cpu_rehearsal.py) to exercise the launcher and the N>1 bookkeeping
without a GPU; its line is marked as a rehearsal and measures nothing.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
SEED = 1896             # RANDOM_SEED, reference src/utils/utils.hpp:26
NSETS = 3               # resident buffer sets in rotation (module doc)

WORKLOADS = {
    # name: (k, m, bs, stripes per GPU, description)
    "cfg3": (16, 1, 1 << 20, 256, "BASELINE configs[2]: k=16+1, 1 MiB shards, enc + single-erasure dec"),
    "cfg2": (8, 1, 1 << 16, 1024, "BASELINE configs[1] shape: k=8+1, 64 KiB shards, 1024 stripes"),
    "cfg4": (32, 1, 4096, 65536, "BASELINE configs[3] shape: k=32+1, 4 KiB shards, 65536 stripes"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="cfg3",
                    help=f"one of {sorted(WORKLOADS)}, or a custom shape k,m,bs,S")
    ap.add_argument("--stripes", type=int, default=0, help="override stripes per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline wall budget")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL (default); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--no-scatter", action="store_true",
                    help="skip the N>1 scatter-inclusive measurement (RCCL send/recv)")
    ap.add_argument("--scatter-timeout", type=float, default=120.0,
                    help="watchdog (s) over the legs after the headline: host pipeline, scatter")
    ap.add_argument("--lost", type=int, default=1,
                    help="lost data blocks per stripe (1..m, one per parity class); the "
                         "BASELINE workloads lose one")
    ap.add_argument("--graph", action="store_true",
                    help="also time the step replayed from one captured hipGraph (needs "
                         "--decode-api device: the host decode scans and copies on the host)")
    ap.add_argument("--decode-api", default="host", choices=["host", "device"],
                    help="host: xec_decode (reference-shaped: host bitmap scan + H2D copy); "
                         "device: xec_decode_device (bitmap resident, verdict on the device)")
    ap.add_argument("--decode-tiling", type=int, default=0, choices=[0, 1, 2, 3],
                    help="xec_set_decode_tiling (diagnostic; 0 = the library's automatic choice)")
    ap.add_argument("--kernel-events", default="dispatch", choices=["dispatch", "packets"],
                    help="per-kernel timing: dispatch = HIP events recorded by each timed "
                         "kernel's own dispatch (xec_set_kernel_events), nothing queued "
                         "between kernels; packets = one hipEventRecord between every two "
                         "kernels (each a queue packet, ~6 us of gap)")
    ap.add_argument("--dist-world1", action="store_true",
                    help="at N=1, still open a one-rank process group (RCCL with nccl) and run "
                         "the collectives and the scatter/gather leg: exercises the N>1 "
                         "communication code on a one-GPU box")
    ap.add_argument("--rehearse-cpu", action="store_true",
                    help="CPU stand-ins for every device call (tools/cpu_rehearsal.py), gloo "
                         "only: rehearses the launcher and N>1 bookkeeping; measures nothing")
    ap.add_argument("--no-host-pipeline", action="store_true",
                    help="skip the host-in/host-out leg (xec_pipeline, pinned host memory)")
    ap.add_argument("--host-stripes", type=int, default=0,
                    help="stripes per rank for the host-in/host-out leg (0 = 1 GiB of data)")
    ap.add_argument("--rehearse-leg-delay", type=float, default=0.0,
                    help="with --rehearse-cpu only: the scatter leg first sleeps this long, so "
                         "a test can make the legs' watchdog fire deterministically")
    ap.add_argument("--rank-grace", type=float, default=60.0,
                    help="launcher: seconds to wait for the other ranks after one fails")
    ap.add_argument("--multi-devices", default="",
                    help="the multi_device leg's device list (comma separated, repeats allowed: "
                         "0,0 rehearses it on one GPU); default at N>1: the N devices the ranks "
                         "ran on; 'none' skips it")
    ap.add_argument("--multi-timeout", type=float, default=300.0,
                    help="seconds before the multi_device leg's child process is killed")
    return ap.parse_args()


def workload_shape(name):
    """A named BASELINE workload, or a custom "k,m,bs,S" (parity-test shapes,
    sweeps); returns (k, m, bs, S, description)."""
    if name in WORKLOADS:
        return WORKLOADS[name]
    try:
        k, m, bs, S = (int(x) for x in name.split(","))
    except ValueError:
        sys.exit(f"--workload: expected one of {sorted(WORKLOADS)} or k,m,bs,S, got {name!r}")
    return k, m, bs, S, f"custom: k={k}+{m}, {bs} B shards, {S} stripes per GPU"


def algorithmic_bytes(S, k, m, bs):
    """encode reads k, writes m blocks per stripe; single-erasure
    decode (one lost data block per stripe) reads k/m - 1 survivors + 1 parity
    and writes 1 block."""
    return S * (k + m) * bs, S * (k // m + 1) * bs


def erasure_pattern(np, S, k, m, lost=1, start=0):
    """Bitmap (S, k+m) of the bench's erasures: one lost data block per stripe at
    (7c) mod k over the global stripe index c; with lost > 1
    (tools), `lost` data blocks per stripe, each in its own parity class
    (class (c+q) mod m, member (7c+q) mod k/m), so every stripe stays
    recoverable (is_recoverable, xorec_utils.hpp:160-175)."""
    c = np.arange(start, start + S)
    bm = np.ones((S, k + m), dtype=np.uint8)
    if lost == 1:
        bm[np.arange(S), (7 * c) % k] = 0
        return bm
    assert 1 <= lost <= m, "lost must be 1..m"
    for q in range(lost):
        bm[np.arange(S), (c + q) % m + m * ((7 * c + q) % (k // m))] = 0
    return bm


def load_traffic(workload):
    """PMC-measured HBM bytes per encode launch, from profiles/ (tools/pmc_traffic.py)."""
    f = ROOT / "profiles" / f"traffic_{workload}.json"
    if not f.exists():
        return None, None
    t = json.loads(f.read_text())
    return t.get("encode_hbm_bytes_per_launch"), t


def rocprof_avg_ns(traffic_src, kernel_base):
    """The rocprofv3 --kernel-trace --stats average (AverageNs) of the kernel
    whose name starts with `kernel_base`, from the kernel-stats CSV that
    profiles/traffic_<workload>.json names as its timing source -- the same
    profiling session as its PMC bytes (tools/pmc_traffic.py).  Returns
    {"avg_ns", "calls", "kernel", "source"} or None (no such file or row)."""
    import csv
    src = (traffic_src or {}).get("timing_source")
    if not src:
        return None
    path = ROOT / src
    if not path.exists():
        return None
    for row in csv.DictReader(open(path)):
        name = row["Name"].split("(")[0].replace("void ", "")
        if name.split("<")[0] == kernel_base:
            return {"avg_ns": float(row["AverageNs"]), "calls": int(row["Calls"]),
                    "kernel": name, "source": src}
    return None


def build_id_of(info):
    """The "src:<id>" token of an xec_build_info() string: the hash of the
    sources the library was built from (erasure-code-benchmark_amd/Makefile)."""
    for tok in (info or "").split():
        if tok.startswith("src:"):
            return tok[4:]
    return None


TIMING_SOURCES = {
    "dispatch": "HIP events recorded by each timed launch's own dispatch (xec_set_kernel_events "
                "-> hipExtLaunchKernel) on the launch stream, every timed launch of this run",
    "packets": "HIP events on the launch stream over the timed region, this run (one "
               "hipEventRecord per kernel boundary: each adds its ~6 us queue-packet gap, "
               "DESIGN.md §4)",
}


def roofline(kernel, b, ms_hip, hbm, traffic_src, lib_build_id=None, timing="dispatch"):
    """SURVEY.md §8(d) roofline of one kernel.  `achieved` = algorithmic bytes
    per launch / the kernel's average launch duration measured live in this
    run with HIP events on the stream it is launched on, over the timed region
    (the contract; VERDICT r05 weak 3: the headline fraction is measured on the
    box that produced the value).  Beside it, `rocprof_profile`: the same
    kernel's rocprofv3 --kernel-trace --stats average (AverageNs) from the
    kernel-stats CSV that profiles/traffic_<workload>.json names -- the profile
    of the same command, committed under profiles/, from the session that
    measured the PMC `traffic` -- so that figure is recomputable from profiles/
    alone, and `over_hip_events_ms` says how well the two clocks agree."""
    hip = b / (ms_hip * 1e-3) / 1e9
    base = kernel.split("<")[0].split(" ")[0]
    prof = rocprof_avg_ns(traffic_src, base)
    r = {"bound": "hbm", "achieved": round(hip, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
         "frac": round(hip / HBM_PEAK_GBPS, 4), "traffic": hbm, "kernel": kernel,
         "algorithmic_bytes_per_launch": b, "avg_launch_ms": round(ms_hip, 4),
         "timing_source": TIMING_SOURCES[timing]}
    if prof:
        pa = b / prof["avg_ns"]  # bytes per ns = GB/s
        r["rocprof_profile"] = {
            "achieved": round(pa, 1), "frac": round(pa / HBM_PEAK_GBPS, 4),
            "avg_launch_ms": round(prof["avg_ns"] * 1e-6, 4), "calls": prof["calls"],
            "kernel": prof["kernel"],
            "source": f"rocprofv3 --kernel-trace --stats AverageNs: {prof['source']}",
            "over_hip_events_ms": round(prof["avg_ns"] * 1e-6 / ms_hip, 4)}
    if traffic_src and hbm is not None:
        r["traffic_source"] = traffic_src.get("source")
    if traffic_src:  # which library the profile measured, and the one this line ran
        r["profile_build_id"] = traffic_src.get("build_id")
        r["library_build_id"] = lib_build_id
        r["profile_is_this_library"] = (lib_build_id is not None and
                                        traffic_src.get("build_id") == lib_build_id)
    return r


def _cpu_model():
    model, avx512 = "", False
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name") and not model:
                model = line.split(":", 1)[1].strip()
            if line.startswith("flags"):
                avx512 = " avx512f" in line
                break
    except OSError:
        pass
    return model, avx512


def _host_threads():
    """(nproc, OMP_NUM_THREADS or None, cgroup CPU quota or None): the CPUs this
    process may run on (its affinity mask, what `nproc` prints), the OpenMP
    thread count the environment asks for (16 on the GPU box, its CPU share),
    and the cgroup v2 cpu.max quota in CPUs when one is set."""
    try:
        nproc = len(os.sched_getaffinity(0))
    except AttributeError:
        nproc = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    return nproc, omp, quota


def cpu_time_port(o, xo, batch, k, m, bs, S, budget_s, threads):
    """The oracle's C restatement of the reference CPU plugin loop
    (XorecBenchmark::encode/decode, xorec_bm.cpp:27-58: OpenMP parallel-for over
    stripes calling xorec_encode / xorec_decode, xorec.cpp:24-111) on one
    resident host batch (`batch` = (data, parity) from o.batch), single erasure
    (7c) mod k per stripe; repeated until `budget_s` of wall time.  Returns
    (GB/s of algorithmic bytes, reps, seconds)."""
    data, parity = batch
    bm = xo.single_erasure_bitmap(S, k, m)
    b_enc, b_dec = algorithmic_bytes(S, k, m, bs)
    reps, t_tot = 0, 0.0
    while (t_tot < budget_s or reps == 0) and reps < 100000:
        t0 = time.perf_counter()
        assert o.encode_batch(data, parity, S, bs, k, m, threads) == 0
        assert o.decode_batch(data, parity, S, bs, k, m, bm, threads) == 0
        t_tot += time.perf_counter() - t0
        reps += 1
    return reps * (b_enc + b_dec) / t_tot / 1e9, reps, t_tot


# Data bytes per CPU sample: every BASELINE shape at its own full batch (config 4:
# 65,536 stripes = 8 GiB), far beyond any host LLC
CPU_SAMPLE_BYTES = 8 << 30
CPU_SAMPLES = 3             # timed samples per figure: median, min and max reported


def parse_cpulist(text):
    """"0-3,8,10-11" (sysfs cpulist) -> [0, 1, 2, 3, 8, 10, 11]."""
    out = []
    for part in text.strip().split(","):
        if part:
            lo, _, hi = part.partition("-")
            out.extend(range(int(lo), int(hi or lo) + 1))
    return out


def cpu_places(threads, numa_node=None, sysfs="/sys", allowed=None):
    """The CPUs the CPU baseline's `threads` OpenMP threads are bound to, one
    each (OMP_PLACES, OMP_PROC_BIND=close): CPUs this process may run on (its
    affinity mask), those on the GPU's NUMA node first, spread round robin
    over the node's L3 domains (CCDs on EPYC: each reaches memory through its
    own link, so 16 threads packed on two CCDs were capped at 132 GB/s where
    the same threads unbound reached 268, profiles/r04e), one CPU per physical
    core before any SMT sibling; the rest of the mask only if the node has too
    few.  So the threads neither migrate nor leave the node whose memory they
    first-touch (the batch is filled in parallel by the same threads)."""
    allowed = sorted(os.sched_getaffinity(0) if allowed is None else allowed)
    node = set()
    if numa_node is not None and numa_node >= 0:
        try:
            node = set(parse_cpulist(Path(f"{sysfs}/devices/system/node/node{numa_node}/cpulist")
                                     .read_text()))
        except OSError:
            node = set()

    def first_of(c, rel):
        try:
            return min(parse_cpulist(Path(f"{sysfs}/devices/system/cpu/cpu{c}/{rel}")
                                     .read_text()))
        except (OSError, ValueError):
            return None

    prim = {c: first_of(c, "topology/thread_siblings_list") in (c, None) for c in allowed}
    l3 = {c: first_of(c, "cache/index3/shared_cpu_list") or 0 for c in allowed}

    def spread(cpus):  # round robin over L3 domains, each domain's CPUs in order
        groups = {}
        for c in cpus:
            groups.setdefault(l3[c], []).append(c)
        lanes = [groups[g] for g in sorted(groups)]
        out = []
        for i in range(max((len(x) for x in lanes), default=0)):
            out += [x[i] for x in lanes if i < len(x)]
        return out

    order = (spread([c for c in allowed if c in node and prim[c]]) +
             spread([c for c in allowed if c in node and not prim[c]]) +
             spread([c for c in allowed if c not in node and prim[c]]) +
             spread([c for c in allowed if c not in node and not prim[c]]))
    return order[:max(1, threads)]


def cpu_measure(spec):
    """Runs in the CPU baseline's child process (bench.py --cpu-baseline-child,
    started by cpu_baseline with the OpenMP binding in its environment, so the
    OpenMP runtime reads it at start-up): CPU_SAMPLES timed samples of each
    figure on one resident batch per shape.  Only this leg imports oracle/."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import xorec_oracle as xo  # the CPU baseline leg is the only bench use of oracle/

    o = xo.COracle()
    threads, budget, nsamp = spec["threads"], spec["budget_s"], spec.get("samples", CPU_SAMPLES)

    def shape(k, m, bs, S_gpu, budget, single_budget):
        S = max(1, min(S_gpu, spec.get("sample_bytes", CPU_SAMPLE_BYTES) // (k * bs)))
        batch = o.batch(S, k, m, bs, threads=threads)  # parallel first touch
        vals, reps, wall = [], 0, 0.0
        for _ in range(nsamp):
            v, r, t = cpu_time_port(o, xo, batch, k, m, bs, S, budget / nsamp, threads)
            vals.append(v)
            reps += r
            wall += t
        res = {"value": round(statistics.median(vals), 2), "unit": "GB/s", "cores": threads,
               "kind": "port", "samples": [round(v, 2) for v in vals],
               "min": round(min(vals), 2), "max": round(max(vals), 2),
               "sample": f"median of {nsamp} samples, {reps} x (encode+decode) in all, of {S} "
                         f"stripes k={k}+{m} {bs >> 10} KiB ({S * k * bs >> 20} MiB data), "
                         f"oracle/xorec_oracle.c (restates xorec.cpp:24-111), OpenMP over "
                         f"stripes as xorec_bm.cpp:30, {threads} threads, {wall:.1f} s wall"}
        if single_budget:
            v1, r1, t1 = cpu_time_port(o, xo, batch, k, m, bs, S, single_budget, 1)
            res["single_thread"] = {"value": round(v1, 2), "unit": "GB/s",
                                    "sample": f"{r1} x the same batch on 1 thread, {t1:.1f} s wall"}
        del batch
        return res

    k, m, bs, S_gpu = spec["k"], spec["m"], spec["bs"], spec["S_gpu"]
    out = shape(k, m, bs, S_gpu, budget, min(2.0, budget) if spec.get("single", True) else 0)
    if spec.get("by_workload"):
        by = {}
        for name, (kk, mm, bb, SS, _) in WORKLOADS.items():
            r = out if name == spec["workload"] else shape(kk, mm, bb, SS, budget / 3, budget / 9)
            by[name] = {kx: r[kx] for kx in ("value", "cores", "min", "max", "single_thread",
                                               "sample")}
        out["by_workload"] = by
    return out


def _cpu_child(spec, env, timeout):
    import subprocess
    p = subprocess.run([sys.executable, str(Path(__file__).resolve()), "--cpu-baseline-child",
                        json.dumps(spec)], capture_output=True, text=True, env=env,
                       timeout=timeout, cwd=str(ROOT))
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        raise RuntimeError(f"CPU baseline child exit {p.returncode}: {p.stderr[-300:]}")
    return json.loads(lines[-1])


PLACEMENTS = {"gpu_node_bound": None, "unbound": "unbound_diagnostic",
              "all_nodes_bound": "all_nodes_diagnostic"}


def pick_best_placement(out):
    """`value` is the FASTEST placement of the same thread count that this run
    measured (BASELINE.md §2 asks for `nproc` threads and no particular
    binding; ADVICE r04: the GPU-node binding alone under-reported the host by
    ~20 %).  The GPU-node-bound figure stays beside it as
    `gpu_node_bound_diagnostic`, every placement's median in `placements`, and
    `placement` names the headline.  by_workload / single_thread stay the
    GPU-node-bound child's (the only one that times them)."""
    cands = {"gpu_node_bound": out}
    for name, key in PLACEMENTS.items():
        d = out.get(key) if key else None
        if isinstance(d, dict) and d.get("value"):
            cands[name] = d
    out["placements"] = {n: d["value"] for n, d in cands.items()}
    best = max(cands, key=lambda n: cands[n]["value"])
    out["placement"] = best
    out["gpu_node_bound_diagnostic"] = {kx: out[kx] for kx in ("value", "min", "max", "samples")}
    if best != "gpu_node_bound":
        d = cands[best]
        for kx in ("value", "min", "max", "samples"):
            out[kx] = d[kx]
        out["sample"] += (f"; value = the {best} placement of the same threads "
                          f"(fastest of {sorted(cands)}), median of its samples")
    return out


def cpu_baseline(workload, k, m, bs, S_gpu, budget_s, numa_node=None,
                 sample_bytes=CPU_SAMPLE_BYTES):
    """BASELINE.md §2 / SURVEY.md §8(d): the CPU XOR-EC path timed on this host's
    cores on a bounded sample of the same workload, as the build's restatement
    (oracle/xorec_oracle.c, "kind": "port"; in-container agreement with the
    reference's own compiled code: profiles/r02_cpu_port_vs_ref.json).

    Threads: the CPUs this process may use -- the smallest of the affinity
    mask, OMP_NUM_THREADS and the cgroup quota (16 on the GPU box: a 16-CPU
    quota over a 256-CPU mask) -- each bound to its own physical core on the
    GPU's NUMA node (cpu_places; OMP_PROC_BIND=close, OMP_PLACES), in a child
    process so the OpenMP runtime starts with that binding: the median of
    CPU_SAMPLES samples (min / max beside it), plus 1 thread and the other
    BASELINE shapes (`by_workload`).  The same threads UNBOUND
    (OMP_PROC_BIND=false: the scheduler free to spread them over the whole
    mask, both sockets) are timed once more as `unbound_diagnostic` -- the
    placement rounds 1-3 ran with -- and bound across every node as
    `all_nodes_diagnostic`.  `value` is the fastest of the three
    (pick_best_placement).  Nothing built from the reference runs here."""
    nproc, omp, quota = _host_threads()
    threads = max(1, min(x for x in (nproc, omp, int(quota) if quota else None) if x))
    cpus = cpu_places(threads, numa_node)
    spec = {"workload": workload, "k": k, "m": m, "bs": bs, "S_gpu": S_gpu,
            "budget_s": budget_s, "threads": threads, "sample_bytes": sample_bytes,
            "samples": CPU_SAMPLES, "by_workload": True}
    base = {kx: v for kx, v in os.environ.items() if not kx.startswith(("OMP_PLACES",
                                                                         "OMP_PROC_BIND",
                                                                         "GOMP_CPU_AFFINITY"))}
    places = ",".join("{%d}" % c for c in cpus)
    env_bound = dict(base, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close", OMP_PLACES=places)
    timeout = 8 * budget_s + 240
    out = _cpu_child(spec, env_bound, timeout)
    out["cpu_model"] = _cpu_model()[0]
    out["nproc"] = nproc
    out["omp_num_threads"] = omp
    out["cgroup_cpu_quota"] = quota
    out["spread_note"] = ("min / max: the spread within this run; value is the fastest of the "
                          "placements timed here (placements); between boxes the GPU-node "
                          "binding measured 266-382 GB/s at cfg3 in round 4 and the placements "
                          "of one box 302-517 in round 5 (which NUMA node holds the GPU, and "
                          "the shared host's other load; DESIGN.md §4)")
    out["binding"] = {"OMP_PROC_BIND": "close", "OMP_PLACES": places, "cpus": cpus,
                      "gpu_numa_node": numa_node,
                      "note": "one thread per physical core of the GPU's NUMA node, spread "
                              "round robin over its L3 domains (CCDs), within the affinity "
                              "mask; threads = min(mask, OMP_NUM_THREADS, cgroup quota)"}
    try:
        free = _cpu_child(dict(spec, by_workload=False, single=False, budget_s=budget_s / 3),
                          dict(base, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="false"),
                          timeout)
        out["unbound_diagnostic"] = {
            kx: free[kx] for kx in ("value", "min", "max", "samples", "cores")}
        out["unbound_diagnostic"]["note"] = (
            "the same threads unbound (OMP_PROC_BIND=false, scheduler places them anywhere in "
            "the mask): the placement of rounds 1-3; bound / unbound = "
            f"{out['value'] / free['value']:.2f}" if free["value"] else "")
    except (RuntimeError, OSError, ValueError) as e:  # diagnostic only
        out["unbound_diagnostic"] = {"error": repr(e)[:200]}
    # The same threads bound one per L3 domain over the WHOLE mask (both
    # sockets on a two-socket box: twice the memory channels, each thread
    # first-touching its own socket's memory) -- what 16 threads of this host
    # can reach, beside the GPU-node figure above
    wide_cpus = cpu_places(threads, None)
    if wide_cpus != cpus:
        try:
            places_all = ",".join("{%d}" % c for c in wide_cpus)
            every = _cpu_child(dict(spec, by_workload=False, single=False, budget_s=budget_s / 3),
                               dict(base, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close",
                                    OMP_PLACES=places_all), timeout)
            out["all_nodes_diagnostic"] = {
                kx: every[kx] for kx in ("value", "min", "max", "samples", "cores")}
            out["all_nodes_diagnostic"]["OMP_PLACES"] = places_all
            out["all_nodes_diagnostic"]["note"] = (
                "the same threads bound one per L3 domain across the whole affinity mask "
                "(every socket), not only the GPU's NUMA node")
        except (RuntimeError, OSError, ValueError) as e:  # diagnostic only
            out["all_nodes_diagnostic"] = {"error": repr(e)[:200]}
    pick_best_placement(out)
    # BASELINE.md §2 names `nproc` threads: where the mask is wider than the
    # CPUs this process may use (256 vs a 16-CPU quota on the GPU box) that
    # count is timed too, unbound, beside the value
    out["by_threads"] = {str(threads): out["value"]}
    if nproc > threads:
        try:
            wide = _cpu_child(dict(spec, by_workload=False, single=False, budget_s=budget_s / 3,
                                   threads=nproc),
                              dict(base, OMP_NUM_THREADS=str(nproc), OMP_PROC_BIND="false"),
                              timeout)
            out["by_threads"][str(nproc)] = wide["value"]
            out["threads_note"] = (f"value at {threads} threads (min of the affinity mask "
                                   f"{nproc}, OMP_NUM_THREADS {omp}, cgroup quota {quota}); "
                                   f"{nproc} threads (nproc) unbound: {wide['value']} GB/s")
        except (RuntimeError, OSError, ValueError) as e:
            out["threads_note"] = f"{nproc} threads (nproc) not timed: {repr(e)[:120]}"
    return out


class DeviceOps:
    """What measure_scatter needs from the device: the HIP path by default;
    tests/test_distributed_cpu.py substitutes CPU stand-ins to run the same
    scatter / encode / gather logic under gloo."""

    def __init__(self, torch, xec, stream, k, m, bs):
        self.torch, self.xec, self.stream = torch, xec, stream
        self.k, self.m, self.bs = k, m, bs
        self.device = "cuda"

    def fill(self, buf, S, seed_base):
        assert self.xec.fill_splitmix64(buf, S, self.k * self.bs, seed_base, self.stream) == 0

    def encode(self, d, p, S):
        assert self.xec.encode(d, p, S, self.bs, self.k, self.m, self.stream) == 0

    def sync(self):
        self.torch.cuda.synchronize()


def measure_scatter(torch, dist, ops, S_total, S, start, k, m, bs, enc_ms, reps=3):
    """Config 5's RCCL legs: the whole batch starts on rank 0,
    is scattered (point-to-point send/recv over xGMI, xec/dist.py), each rank
    encodes its slice, and the parity is gathered back to rank 0, where it must
    equal rank 0's own encode of the whole batch.  Link-bound, so reported
    beside -- never as -- the device-resident value.  `ops` = DeviceOps."""
    from xec import dist as xdist
    from xec import stripe_range
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = ops.device

    def timed(fn):
        ts = []
        for _ in range(reps):
            dist.barrier()
            ops.sync()
            t0 = time.perf_counter()
            fn()
            ops.sync()
            ts.append(time.perf_counter() - t0)
        t = torch.tensor([min(ts)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.item()

    def all_true(flag):
        t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return t.item() == 1.0

    full = torch.empty(S_total * k * bs if rank == 0 else 1, dtype=torch.uint8, device=dev)
    if rank == 0:
        ops.fill(full, S_total, SEED)
    local = torch.empty(S * k * bs, dtype=torch.uint8, device=dev)
    t_sc = timed(lambda: xdist.scatter_stripes(full if rank == 0 else None, local, S_total,
                                               k * bs))
    ref = torch.empty_like(local)
    ops.fill(ref, S, SEED + start)
    ok_sc = all_true(torch.equal(ref, local))
    del ref
    # per-rank encode of the scattered slice, parity gathered back to the root
    lp = torch.empty(S * m * bs, dtype=torch.uint8, device=dev)
    ops.encode(local, lp, S)
    fullp = torch.empty(S_total * m * bs if rank == 0 else 1, dtype=torch.uint8, device=dev)
    t_ga = timed(lambda: xdist.gather_stripes(lp, fullp if rank == 0 else None, S_total, m * bs))
    ok_ga = True
    if rank == 0:
        refp = torch.empty_like(fullp)
        ops.encode(full, refp, S_total)
        ok_ga = bool(torch.equal(refp, fullp))
        del refp
    ok_ga = all_true(ok_ga)
    del full, local, lp, fullp
    a0, b0 = stripe_range(S_total, 0, world)
    remote = S_total - (b0 - a0)  # stripes that cross a link
    return {"bit_exact": ok_sc, "scatter_ms": round(t_sc * 1e3, 3),
            "root_egress_GBps": round(remote * k * bs / t_sc / 1e9, 1),
            "scatter_inclusive_encode_GBps_data": round(
                S_total * k * bs / (t_sc + enc_ms * 1e-3) / 1e9, 1),
            "gather_parity_ms": round(t_ga * 1e3, 3),
            "root_ingress_GBps": round(remote * m * bs / t_ga / 1e9, 1),
            "scatter_encode_gather_GBps_data": round(
                S_total * k * bs / (t_sc + enc_ms * 1e-3 + t_ga) / 1e9, 1),
            "gathered_parity_bit_exact_vs_root_encode": ok_ga,
            "note": f"batch starts on rank 0; {dist.get_backend()} send/recv of stripe ranges "
                    "(RCCL with nccl); link-bound; path = how rank 0's GPU reaches the "
                    "others (topology: xgmi-p2p = peer access over xGMI, staged = none)"}


def scatter_topology(devices, rehearse=False):
    """Config 5's root -> peer pairs as the runtime reports them (xec/topology.py;
    VERDICT r05 item 2): rank 0's device is the root, `devices` the ranks'
    devices.  A CPU rehearsal has no runtime to ask: it records the
    XEC_TOPOLOGY_STUB topology, or says it has none."""
    from xec import topology
    if rehearse and not os.environ.get("XEC_TOPOLOGY_STUB"):
        return {"skipped": "CPU rehearsal: no runtime to ask (set XEC_TOPOLOGY_STUB)"}
    try:
        return topology.record(int(devices[0]), [int(d) for d in devices])
    except Exception as e:  # noqa: BLE001 - a diagnostic field, never the line
        return {"error": repr(e)[:200]}


HOST_CHUNK_STRIPES, HOST_STREAMS = 8, 3  # best measured pipeline shape


def gpu_numa_node(torch, dev, sysfs="/sys"):
    """The NUMA node of this rank's GPU (its PCI function in sysfs), for the
    host leg's per-rank record: on a two-socket 8-GPU node half the GPUs hang
    off each socket. HIP already places pinned host allocations on the node
    nearest the current device (hipHostMalloc without hipHostMallocNumaUser),
    so nothing is rebound here; the line shows where each rank's link ends.
    Returns {"numa_node": n}, or a "skipped" reason."""
    try:
        pr = torch.cuda.get_device_properties(dev)
        bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        node = int(Path(f"{sysfs}/bus/pci/devices/{bdf}/numa_node").read_text())
        if node < 0:
            return {"skipped": f"no NUMA node for {bdf}"}
        return {"numa_node": node}
    except (OSError, ValueError, AttributeError) as e:
        return {"skipped": repr(e)[:120]}


def measure_host_pipeline(torch, dist, xec, k, m, bs, S, start, coll_dev, reps=3, pinned=True):
    """North star's end-to-end rate: each rank
    streams a batch that starts and ends in its own host memory -- pinned, or
    with pinned=False pageable like a file or socket buffer -- through
    its GPU with xec_pipeline (H2D -> kernel -> D2H, chunks over streams), all
    ranks at once between barriers.  Encode returns the parity to the host;
    decode rebuilds one lost data block per stripe in host memory.  Returns this
    rank's (encode s, decode s, bit-exact, error, GPU NUMA node); every rank makes the same
    collective calls whatever fails locally.  PCIe-bound: reported beside, never
    as, the device-resident value."""
    import numpy as np
    use_dist = dist.is_initialized()

    def agree(flag):
        if not use_dist:
            return flag
        t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return t.item() == 1.0

    err = None
    numa = gpu_numa_node(torch, torch.cuda.current_device())
    try:  # setup: host batch, its parity and an erasure pattern
        h_d = torch.empty(S * k * bs, dtype=torch.uint8)
        h_p = torch.empty(S * m * bs, dtype=torch.uint8)
        if pinned:
            h_d, h_p = h_d.pin_memory(), h_p.pin_memory()
        d_d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        d_p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        st = torch.cuda.current_stream()
        assert xec.fill_splitmix64(d_d, S, k * bs, SEED + start, st) == 0
        assert xec.encode(d_d, d_p, S, bs, k, m, st) == 0
        h_d.copy_(d_d)
        ref_p = d_p.cpu()
        ref_d = h_d.clone()
        del d_d, d_p
        bm = erasure_pattern(np, S, k, m, 1, start)
        h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
        hv = h_d.numpy().reshape(S, k, bs)
        pl = xec.Pipeline(HOST_CHUNK_STRIPES, bs, k, m, HOST_STREAMS)
    except Exception as e:  # noqa: BLE001 - reported in the line
        err = repr(e)[:200]
    if not agree(err is None):
        return 0.0, 0.0, False, err or "another rank failed its setup", numa

    rcs = []

    def timed(fn, before=None):
        ts = []
        for _ in range(reps + 1):  # the first is a warm-up
            if before is not None:
                before()
            if use_dist:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rcs.append(int(fn()))
            ts.append(time.perf_counter() - t0)
        return min(ts[1:])

    def erase():
        hv[bm[:, :k] == 0] = 0

    h_p.zero_()
    t_enc = timed(lambda: pl.encode(h_d, h_p, S))
    ok = bool(torch.equal(h_p, ref_p))
    t_dec = timed(lambda: pl.decode(h_d, h_p, S, h_bm), before=erase)
    ok &= bool(torch.equal(h_d, ref_d)) and not any(rcs)
    pl.close()
    return (t_enc, t_dec, ok, (f"xec_pipeline status {sorted(set(rcs))}" if any(rcs) else None),
            numa)


MULTI_LEG_BIN = ROOT / "erasure-code-benchmark_amd" / "bin" / "xec_multi_leg"


def multi_device_list(args, world, ndev):
    """The multi_device leg's devices: --multi-devices, else at N > 1 the N
    devices the ranks ran on (rank r on device r % visible, as run_rank picks
    them); None when the leg is off (N = 1 without the flag, or 'none')."""
    spec = args.multi_devices.strip().lower()
    if spec == "none":
        return None
    if spec:
        return [int(x) for x in spec.split(",")]
    if world > 1:
        return [r % ndev for r in range(world)]
    return None


def run_multi_device_leg(args, devices, k, m, bs, S_per):
    """Config 5 through the ONE-process multi-device plugin:
    XorecBenchmarkHipMulti over `devices` -- device-resident encode + decode
    timed from first launch to last completion, validated, then the batch
    scattered from the root's HBM with hipMemcpyPeerAsync, encoded per shard
    and the parity gathered back and compared with the root's own encode
    (host/xec_multi_leg.cpp).  Runs as a fresh child process started after
    every rank has finished its GPU work, under its own time limit: a stuck
    peer copy costs this field, never the line.  With --rehearse-cpu the child
    is the CPU stand-in (tools/cpu_rehearsal.py multi-leg)."""
    import subprocess
    leg_args = ["--devices", ",".join(map(str, devices)), "--stripes-per-device", str(S_per),
                "--data", str(k), "--parity", str(m), "--block", str(bs)]
    if args.rehearse_cpu:
        cmd = [sys.executable, str(ROOT / "tools" / "cpu_rehearsal.py"), "multi-leg", *leg_args]
    else:
        if not MULTI_LEG_BIN.exists():
            return {"error": f"{MULTI_LEG_BIN.relative_to(ROOT)} not built (make -C "
                             "erasure-code-benchmark_amd)"}
        cmd = [str(MULTI_LEG_BIN), *leg_args]
    t0 = time.perf_counter()
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=args.multi_timeout,
                           cwd=str(ROOT))
    except subprocess.TimeoutExpired:
        return {"error": f"timed out ({args.multi_timeout:.0f} s): child killed",
                "devices": devices}
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    try:
        res = json.loads(lines[-1])
    except (IndexError, ValueError):
        res = {"error": f"exit {p.returncode}, no result line; stderr: {p.stderr[-300:]}"}
    if p.returncode != 0 and "error" not in res:
        res["error"] = f"exit {p.returncode} (a check failed: see bit_exact / scatter)"
    res["child_wall_s"] = round(time.perf_counter() - t0, 2)
    res["command"] = " ".join([Path(cmd[0]).name, *cmd[1:]])
    return res


def host_side_wait(dist, rank, key, timeout_s):
    """The other ranks wait for rank 0 on the host, through the process
    group's own rendezvous store (the TCPStore every rank is already
    connected to): rank 0 sets `key`, the others block on it.  An RCCL barrier
    here would keep a collective kernel spinning on every GPU while rank 0's
    multi_device child times them, and a new gloo group would open fresh
    connections at the end of the run.  Falls back to dist.barrier() where the
    store is not reachable."""
    import datetime
    try:
        store = dist.distributed_c10d._get_default_store()
    except (AttributeError, RuntimeError, ValueError):
        store = None
    if store is None:
        dist.barrier()
        return
    if rank == 0:
        store.set(key, "1")
    else:
        store.wait([key], datetime.timedelta(seconds=timeout_s))


def launch_ranks(n, argv, grace_s):
    """`bench.py --gpus N` with no launcher around it: start N rank processes of
    this same script (one per GPU, LOCAL_RANK = device), the environment
    torch.distributed.run would give them, rendezvous on 127.0.0.1.  Runs
    before anything imports torch or touches a GPU; children are started, not
    exec'd.  Rank 0 prints the JSON line; the others print nothing on stdout.
    Exit status: 0 when every rank exits 0; 3 when the ranks exited 0 or 3
    and at least one 3 -- the legs' watchdog fired after rank 0 printed the
    line, whose "host_pipeline" / "scatter" field carries the error -- so a
    hung leg is visible to whoever runs `bench.py --gpus N`; else the first
    failing rank's status, after the others are given `grace_s` and then killed
    (by PID: only the processes started here)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), XEC_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, "-u", str(Path(__file__).resolve()), *argv],
                                      env=env, cwd=str(ROOT)))
    rcs = [None] * n
    t_fail = None
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if t_fail is None and any(rc not in (None, 0, 3) for rc in rcs):
            t_fail = time.monotonic()
        if t_fail is not None and time.monotonic() - t_fail > grace_s:
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.kill()
                    rcs[i] = p.wait()
        time.sleep(0.05)
    bad = [(i, rc) for i, rc in enumerate(rcs) if rc not in (0, 3)]
    if bad:
        print(f"bench.py launcher: rank exit statuses {rcs}", file=sys.stderr)
        rc = bad[0][1]
        return rc if rc > 0 else 1
    if 3 in rcs:
        print(f"bench.py launcher: the legs' watchdog fired on ranks "
              f"{[i for i, rc in enumerate(rcs) if rc == 3]} (the line's host_pipeline / "
              "scatter error says which leg)", file=sys.stderr)
        return 3
    return 0


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--cpu-baseline-child":
        # the CPU baseline's child (cpu_baseline): CPU only, no torch, no GPU
        print(json.dumps(cpu_measure(json.loads(sys.argv[2]))), flush=True)
        return
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.rank_grace))
    run_rank(args)


def _result_stream():
    """The one JSON line goes to the process's stdout; everything else written
    to fd 1 from here on -- RCCL prints a version banner there at communicator
    init, once per rank -- is sent to stderr, so stdout carries exactly the
    result line at any N."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def run_rank(args):
    result_out = _result_stream()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    backend = args.dist_backend
    if args.rehearse_cpu:
        # explicit CPU rehearsal of the launcher / N>1 bookkeeping -- never a fallback
        if backend != "gloo":
            sys.exit("--rehearse-cpu needs --dist-backend gloo")
        if args.graph:
            sys.exit("--graph needs the GPU")
        sys.path.insert(0, str(ROOT / "tools"))
        from cpu_rehearsal import CpuCuda, CpuXec
        xec, cuda, devname = CpuXec(), CpuCuda(), "cpu"
    else:
        import xec
        cuda, devname = torch.cuda, "cuda"
    # rocprofv3 --selected-regions collects only inside markers.timed_region
    # (the timed steps); nothing before it, so warm-up and setup stay out
    from xec import markers
    markers.pause()
    ndev = max(cuda.device_count(), 1)  # does not initialise the GPU on this image
    if backend == "nccl" and world > ndev:
        sys.exit(f"--gpus {world} with RCCL needs {world} visible GPUs, found {ndev} "
                 "(RCCL refuses two ranks on one device; --dist-backend gloo rehearses)")
    # one process per GPU; the modulo only matters when rehearsing N>1 on
    # fewer GPUs under gloo
    dev = local % ndev
    cuda.set_device(dev)
    st = xec.init(dev)
    if st != 0:
        sys.exit(f"xec_init({dev}) failed: {st!r}")
    if args.decode_tiling and xec.set_decode_tiling(args.decode_tiling) != 0:
        sys.exit(f"--decode-tiling {args.decode_tiling} rejected")
    use_dist = world > 1 or args.dist_world1
    if use_dist:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev),
                                    **({} if world > 1 else {
                                        "init_method": f"tcp://127.0.0.1:{_free_port()}",
                                        "rank": 0, "world_size": 1}))
        else:
            dist.init_process_group("gloo", **({} if world > 1 else {
                "init_method": f"tcp://127.0.0.1:{_free_port()}", "rank": 0, "world_size": 1}))
        ranks_seen = dist.get_world_size()
        assert ranks_seen == world, f"process group has {ranks_seen} ranks, expected {world}"
    coll_dev = devname if backend == "nccl" else "cpu"

    k, m, bs, S_per, desc = workload_shape(args.workload)
    if args.stripes:
        S_per = args.stripes
    S_total = S_per * world
    start, stop = xec.stripe_range(S_total, rank, world)
    S = stop - start
    stream = cuda.current_stream()

    # ---- resident inputs: NSETS buffer sets, filled and encoded on the device --
    sets = []
    for s in range(NSETS):
        d = torch.empty(S * k * bs, dtype=torch.uint8, device=devname)
        p = torch.empty(S * m * bs, dtype=torch.uint8, device=devname)
        seed_base = SEED + start + s * (1 << 40)
        assert xec.fill_splitmix64(d, S, k * bs, seed_base, stream) == 0
        assert xec.encode(d, p, S, bs, k, m, stream) == 0
        sets.append((d, p, seed_base))
    # single erasure per stripe, (7c) mod k over the GLOBAL stripe index
    import numpy as np
    bm = erasure_pattern(np, S, k, m, args.lost, start)
    h_bm = torch.from_numpy(bm.reshape(-1))
    if devname == "cuda":
        h_bm = h_bm.pin_memory()
    d_bm = h_bm.to(devname) if devname == "cuda" else h_bm.clone()
    scratch = [torch.empty_like(d_bm) for _ in range(NSETS)]
    d_status = torch.zeros((NSETS,), dtype=torch.int32, device=devname)
    # The lost block's content on entry to decode is irrelevant (include/xec.h),
    # so the timed loop does not re-erase: every decode still reads k/m-1
    # survivors + parity and rewrites the lost block.  Erasure + rebuild is
    # verified for real after the timed region.
    cuda.synchronize()

    # Per-kernel timing, on the stream the kernels are launched on.  Default
    # ("dispatch"): every timed encode / decode records a start and a stop HIP
    # event from its own dispatch (xec_set_kernel_events -> hipExtLaunchKernel),
    # so the timed region queues nothing but the kernels and each interval is
    # that kernel's execution alone.  "packets": ONE hipEventRecord between
    # every two kernels (2K+1 in all), each a queue packet of its own with
    # ~6 us of gap in the kernel trace (tools/lab/event_cost.py,
    # profiles/r05s): events[2i] -> [2i+1] brackets step i's encode,
    # [2i+1] -> [2i+2] its decode.
    dispatch_events = args.kernel_events == "dispatch"

    def step(i, ev=None, stream=stream):
        de, pe, _ = sets[i % NSETS]
        di = (i + NSETS - 1) % NSETS  # the set encoded two kernels ago (module doc)
        dd, pd, _ = sets[di]
        if ev is not None and dispatch_events:
            xec.set_kernel_events(ev[0], ev[1])
        rc = xec.encode(de, pe, S, bs, k, m, stream)
        if ev is not None and not dispatch_events:
            ev[0].record(stream)
        if ev is not None and dispatch_events:
            xec.set_kernel_events(ev[2], ev[3])
        if args.decode_api == "device":
            rc |= xec.decode_device(dd, pd, S, bs, k, m, d_bm, d_status[di:], stream)
        else:
            rc |= xec.decode(dd, pd, S, bs, k, m, h_bm, scratch[di], stream)
        if ev is not None and not dispatch_events:
            ev[1].record(stream)
        return rc

    for i in range(args.warmup):
        assert step(i) == 0
    if dispatch_events:
        events = [cuda.Event(enable_timing=True) for _ in range(4 * args.steps)]
        for e in events:  # torch creates an event's HIP handle at its first record
            e.record(stream)
        cuda.synchronize()
    else:
        events = [cuda.Event(enable_timing=True) for _ in range(2 * args.steps + 1)]

    if use_dist:
        dist.barrier()
    cuda.synchronize()
    t0 = time.perf_counter()
    rc = 0
    with markers.timed_region("bench:timed"):
        if dispatch_events:
            for i in range(args.steps):
                rc |= step(args.warmup + i, events[4 * i:4 * i + 4])
        else:
            events[0].record(stream)
            for i in range(args.steps):
                rc |= step(args.warmup + i, events[2 * i + 1:2 * i + 3])
        cuda.synchronize()
    t1 = time.perf_counter()
    if use_dist:
        dist.barrier()
    assert rc == 0, "xec call failed inside the timed region"
    if args.decode_api == "device":
        assert d_status.tolist() == [0] * NSETS, f"device decode verdicts {d_status.tolist()}"
    elapsed = t1 - t0
    if dispatch_events:
        enc_list = [events[4 * i].elapsed_time(events[4 * i + 1]) for i in range(args.steps)]
        dec_list = [events[4 * i + 2].elapsed_time(events[4 * i + 3]) for i in range(args.steps)]
    else:
        enc_list = [events[2 * i].elapsed_time(events[2 * i + 1]) for i in range(args.steps)]
        dec_list = [events[2 * i + 1].elapsed_time(events[2 * i + 2]) for i in range(args.steps)]
    enc_ms = sum(enc_list) / args.steps
    dec_ms = sum(dec_list) / args.steps

    # ---- optional: the same steps replayed from one captured hipGraph ----------
    # (xec_decode_device has no host work, so a whole rotation of NSETS steps --
    # 2*NSETS kernels plus the decode's status memsets and check kernels -- is
    # one graph; reported beside the headline, never as it)
    graph = None
    if args.graph:
        if args.decode_api != "device":
            sys.exit("--graph needs --decode-api device")
        side = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=side):
            cs = torch.cuda.current_stream()
            for i in range(NSETS):
                assert step(i, stream=cs) == 0
        reps = max(1, args.steps // NSETS)
        g.replay()
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()
        tg0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        tg = time.perf_counter() - tg0
        assert d_status.tolist() == [0] * NSETS, f"graph decode verdicts {d_status.tolist()}"
        graph = {"ms_per_step": round(tg / (reps * NSETS) * 1e3, 4), "steps": reps * NSETS,
                 "note": "one captured rotation of steps replayed; rank-local wall clock"}
        del g

    # ---- correctness of what was timed -------------------------------------
    # parity == XOR of each class's data (encode), then erase -> decode ->
    # data == a fresh device fill (decode); all on the device, no oracle.
    ok = True
    if not args.no_verify:
        fresh = torch.empty_like(sets[0][0])
        for i, (d, p, seed_base) in enumerate(sets):
            blocks = d.view(S, k // m, m, bs).view(torch.int64)
            red = blocks[:, 0]
            for r in range(1, k // m):
                red = torch.bitwise_xor(red, blocks[:, r])
            ok &= bool(torch.equal(red.view(torch.uint8).reshape(-1), p))
            del blocks, red
            assert xec.erase(d, p, S, bs, k, m, d_bm, stream) == 0
            assert xec.fill_splitmix64(fresh, S, k * bs, seed_base, stream) == 0
            ok &= not bool(torch.equal(fresh, d)) or S == 0  # erasure really removed data
            assert xec.decode(d, p, S, bs, k, m, h_bm, scratch[i], stream) == 0
            ok &= bool(torch.equal(fresh, d))
        del fresh

    # which decode kernel xec_decode's tiling launched (xec_decode_tiling_used)
    if args.decode_api == "device":
        dec_kernel = "xec::decode_kernel (xec_decode_device)"
    elif hasattr(xec, "decode_tiling_used"):
        dec_kernel = xec.DECODE_KERNELS.get(xec.decode_tiling_used(), "xec::decode_kernel")
    else:  # CPU rehearsal stand-ins
        dec_kernel = "xec::decode_kernel"
    # every rank's (elapsed, encode ms, decode ms, failed, stripes); rank 0 reports
    # the max time over ranks and each rank's own rates
    # which device this rank ran on (PCI bus id), so the line shows N distinct GPUs
    bus = -1.0
    if devname == "cuda":
        bus = float(getattr(torch.cuda.get_device_properties(dev), "pci_bus_id", -1))
    mine = torch.tensor([elapsed, enc_ms, dec_ms, 0.0 if ok else 1.0, float(S), float(dev), bus],
                        dtype=torch.float64, device=coll_dev)
    if use_dist:
        rows = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(rows, mine)
        rows = [r.tolist() for r in rows]
    else:
        rows = [mine.tolist()]
    elapsed = max(r[0] for r in rows)
    enc_ms_max = max(r[1] for r in rows)
    dec_ms_max = max(r[2] for r in rows)
    bad = max(r[3] for r in rows)
    stripes_done = int(sum(r[4] for r in rows))

    b_enc, b_dec = algorithmic_bytes(S_per, k, m, bs)  # per GPU
    b_dec *= args.lost
    # all ranks' algorithmic bytes (ranges may be ragged only with --stripes
    # and S_total < world, never at the BASELINE shapes)
    e_all, d_all = algorithmic_bytes(stripes_done, k, m, bs)
    total_bytes = args.steps * (e_all + d_all * args.lost)
    value = total_bytes / elapsed / 1e9
    if rank == 0:
        traffic, traffic_src = load_traffic(args.workload)
        if traffic_src and traffic_src.get("encode_algorithmic_bytes_per_launch") != b_enc:
            traffic, traffic_src = None, None  # profiled at another batch size (--stripes)
        traffic_dec = traffic_src.get("decode_hbm_bytes_per_launch") if traffic_src else None
        if traffic_src and args.lost != 1:
            traffic_src, traffic, traffic_dec = None, None, None  # profiled at one erasure
        # the dominant kernel is the one the step spends longer in (decode at the
        # BASELINE shapes: in-place writes); both are reported
        lib_id = build_id_of(xec.build_info()) if not args.rehearse_cpu else None
        rl = {"encode": roofline("xec::encode_kernel", b_enc, enc_ms, traffic, traffic_src, lib_id,
                                 args.kernel_events),
              "decode": roofline(dec_kernel, b_dec, dec_ms, traffic_dec, traffic_src, lib_id,
                                 args.kernel_events)}
        dominant = ("decode" if rl["decode"]["avg_launch_ms"] >= rl["encode"]["avg_launch_ms"]
                    else "encode")
        cpu = None
        if world == 1 and not args.no_cpu_baseline and args.lost == 1 and not args.rehearse_cpu:
            numa = gpu_numa_node(torch, dev) if devname == "cuda" else {}
            cpu = cpu_baseline(args.workload, k, m, bs, S_per, args.cpu_seconds,
                               numa.get("numa_node"))
        metric = json.loads((ROOT / "BASELINE.json").read_text())["metric"]
        out = {
            "metric": metric,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": ("CPU REHEARSAL of the launcher and N>1 bookkeeping (tools/cpu_rehearsal.py):"
                     " not a measurement" if args.rehearse_cpu else
                     "synthetic: splitmix64 u64 words, stripe seed 1896+global stripe; "
                     "generated in HBM"),
            "config": {"workload": f"{args.workload}: {desc}", "k": k, "m": m, "block_bytes": bs,
                       "stripes_per_gpu": S_per, "stripes_total": S_total,
                       "erasure": "data block (7c) mod k lost per stripe" if args.lost == 1 else
                       f"{args.lost} data blocks lost per stripe, one per parity class",
                       "parallelism": f"stripe-partition x{world} (no data-path collective)",
                       "bytes_convention": "algorithmic: enc S(k+m)bs + dec S(k/m+1)bs",
                       "decode_api": "xec_decode_device" if args.decode_api == "device"
                       else "xec_decode",
                       "decode_tiling": args.decode_tiling or "automatic",
                       "kernel_timing": args.kernel_events},
            "roofline": dict(rl[dominant], dominant_by="avg launch time (avg_launch_ms)"),
            # north star: the device-resident rate at every N also as a fraction of
            # the HBM roofline of the N GPUs together (value / (N x 8 TB/s))
            "value_frac_of_n_gpu_hbm_peak": round(value / (world * HBM_PEAK_GBPS), 4),
            "roofline_by_kernel": rl,
            "cpu_baseline": cpu,
            "encode_ms": round(enc_ms_max, 4),
            "decode_ms": round(dec_ms_max, 4),
            "encode_GBps_per_gpu": round(b_enc / (enc_ms_max * 1e-3) / 1e9, 1),
            "decode_GBps_per_gpu": round(b_dec / (dec_ms_max * 1e-3) / 1e9, 1),
            "data_GBps_reference_convention": round(
                2 * args.steps * stripes_done * k * bs / elapsed / 1e9, 2),
            "verified": bad == 0.0,
            "graph": graph,
            "dist": {"backend": dist.get_backend() if use_dist else None,
                     "ranks_seen": dist.get_world_size() if use_dist else 1,
                     "launcher": "bench.py" if os.environ.get("XEC_BENCH_SPAWNED") else
                     ("external" if world > 1 else None)},
            # each rank's own HIP-event launch rates (weak scaling: same S per rank)
            "per_rank": [{"rank": i, "stripes": int(r[4]),
                          "encode_GBps": round(algorithmic_bytes(int(r[4]), k, m, bs)[0]
                                               / (r[1] * 1e-3) / 1e9, 1) if r[1] else None,
                          "decode_GBps": round(args.lost * algorithmic_bytes(int(r[4]), k, m, bs)[1]
                                               / (r[2] * 1e-3) / 1e9, 1) if r[2] else None,
                          "elapsed_ms": round(r[0] * 1e3, 3), "device": int(r[5]),
                          "pci_bus_id": int(r[6])} for i, r in enumerate(rows)],
            # per-launch HIP-event statistics on rank 0 (median with stddev)
            "launch_stats_rank0": {
                n: {"mean_ms": round(statistics.fmean(v), 4),
                    "median_ms": round(statistics.median(v), 4),
                    "stdev_ms": round(statistics.stdev(v), 4) if len(v) > 1 else 0.0,
                    "min_ms": round(min(v), 4), "max_ms": round(max(v), 4)}
                for n, v in (("encode", enc_list), ("decode", dec_list))},
            # the same launches by resident buffer set: where a set's pages sit in
            # HBM moves its rate by a few % (DESIGN.md §3 *Placement*); step i
            # encodes set i % NSETS and decodes set (i + NSETS - 1) % NSETS
            "median_ms_by_set_rank0": {
                n: [round(statistics.median(
                    [t for i, t in enumerate(v) if (args.warmup + i + shift) % NSETS == q]), 4)
                    if args.steps >= NSETS else None for q in range(NSETS)]
                for n, v, shift in (("encode", enc_list, 0), ("decode", dec_list, NSETS - 1))},
        }
        if use_dist:
            # how the scatter leg's bytes travel from rank 0's GPU to each rank's
            # (a CPU rehearsal stands for an N-GPU node: rank r on device r)
            out["topology"] = scatter_topology(
                list(range(world)) if args.rehearse_cpu else [int(r[5]) for r in rows],
                args.rehearse_cpu)
    else:
        out = None

    # Two legs run after the headline numbers are final, under one watchdog: a
    # stuck link or copy can cost their fields, never the result line.  On
    # expiry every rank exits 3 (rank 0 prints the line first, with the leg's
    # "error"), at any N: a plain `python bench.py` as well as the bench.py
    # launcher and an external one return 3 -- "headline printed, a leg hung"
    # (tests/test_bench_launcher.py).
    #  * host_pipeline: the north star's host-in / host-out rate, every rank;
    #  * scatter: config 5's RCCL scatter / gather (N > 1; gloo cannot carry
    #    HIP buffers, so with --dist-backend gloo on a GPU it is skipped).
    host_leg = not args.no_host_pipeline and not args.rehearse_cpu and args.lost == 1 and not bad
    scatter_leg = (use_dist and not args.no_scatter and not bad
                   and (backend == "nccl" or args.rehearse_cpu))
    if host_leg or scatter_leg:
        import threading

        # Each leg's result is merged into the line under `lock`; the watchdog
        # prints the line under the same lock and marks it printed, so it never
        # serialises `out` while a leg is being added, and a leg that finishes
        # after it changes nothing.  rocprofv3 --marker-trace shows each leg as
        # a ROCTx range (the headline launches are bench:timed).
        lock = threading.Lock()
        printed = []

        def merge(leg, value):
            with lock:
                if out is not None and not printed:
                    out[leg] = value

        def on_timeout():
            with lock:
                if printed:  # the legs finished while the timer was firing
                    return
                if out is not None:
                    for leg, on in (("host_pipeline", host_leg), ("scatter", scatter_leg)):
                        if on and leg not in out:
                            out[leg] = {"error": f"timed out ({args.scatter_timeout:.0f} s watchdog)"}
                    print(json.dumps(out), file=result_out, flush=True)
                printed.append(True)
            sys.stderr.flush()
            os._exit(3)

        dog = threading.Timer(args.scatter_timeout, on_timeout)
        dog.daemon = True
        dog.start()
        if host_leg:
            hs = args.host_stripes or max(1, (1 << 30) // (k * bs))
            with markers.region("bench:host_pipeline"):
                t_enc, t_dec, ok_h, err, numa = measure_host_pipeline(
                    torch, dist, xec, k, m, bs, hs, start, coll_dev)
                # the same from pageable buffers (file / socket buffers)
                pg_enc, pg_dec, ok_pg, err_pg, _ = measure_host_pipeline(
                    torch, dist, xec, k, m, bs, hs, start, coll_dev, pinned=False)
            err = err or err_pg
            mine = torch.tensor([t_enc, t_dec, 1.0 if ok_h else 0.0,
                                 float(numa.get("numa_node", -1)), pg_enc, pg_dec,
                                 1.0 if ok_pg else 0.0], dtype=torch.float64, device=coll_dev)
            if use_dist:
                hrows = [torch.zeros_like(mine) for _ in range(world)]
                dist.all_gather(hrows, mine)
                hrows = [r.tolist() for r in hrows]
            else:
                hrows = [mine.tolist()]
            te, td = max(r[0] for r in hrows), max(r[1] for r in hrows)
            data_all = world * hs * k * bs
            hp = {"encode_GBps_data": round(data_all / te / 1e9, 2) if te > 0 else None,
                  "decode_GBps_data": round(data_all / td / 1e9, 2) if td > 0 else None,
                  "bit_exact": all(r[2] == 1.0 for r in hrows),
                  "per_rank_encode_GBps_data": [
                      round(hs * k * bs / r[0] / 1e9, 2) if r[0] else None for r in hrows],
                  # the NUMA node each rank's GPU hangs off (-1: sysfs names none)
                  "per_rank_numa_node": [int(r[3]) for r in hrows],
                  "pageable": {
                      "encode_GBps_data": round(data_all / max(r[4] for r in hrows) / 1e9, 2)
                      if all(r[4] > 0 for r in hrows) else None,
                      "decode_GBps_data": round(data_all / max(r[5] for r in hrows) / 1e9, 2)
                      if all(r[5] > 0 for r in hrows) else None,
                      "bit_exact": all(r[6] == 1.0 for r in hrows),
                      "note": "the same batch in pageable host memory (file / socket buffers)"},
                  "sample": f"{hs} stripes ({hs * k * bs >> 20} MiB data) per rank in pinned "
                            f"host memory, xec_pipeline {HOST_CHUNK_STRIPES}-stripe chunks x "
                            f"{HOST_STREAMS} streams, all ranks at once, best of 3 after a "
                            "warm-up, max over ranks; encode = data in, parity out; decode "
                            "= survivors in, one rebuilt block per stripe out",
                  "note": "end-to-end, PCIe-bound (DESIGN.md §7); reported beside the "
                          "device-resident value, never as it"}
            if "skipped" in numa:
                hp["numa_rank%d" % rank] = numa["skipped"]
            if err:
                hp["error"] = err
                print(f"rank {rank}: host_pipeline: {err}", file=sys.stderr)
            merge("host_pipeline", hp)
        if scatter_leg:
            try:
                ops = DeviceOps(torch, xec, stream, k, m, bs)
                ops.device, ops.sync = coll_dev, cuda.synchronize
                if args.rehearse_cpu and args.rehearse_leg_delay > 0:
                    time.sleep(args.rehearse_leg_delay)  # a stuck link, rehearsed
                with markers.region("bench:scatter"):
                    sc = measure_scatter(torch, dist, ops, S_total, S, start, k, m, bs, enc_ms)
            except Exception as e:  # noqa: BLE001 - report, keep the headline line
                sc = {"error": repr(e)[:200]}
            if out is not None:  # rank 0: xgmi-p2p, staged, ... from the topology record
                sc["path"] = out.get("topology", {}).get("path", "unknown")
            merge("scatter", sc)
        with lock:
            printed.append(True)  # a watchdog firing from here on finds the legs done
        dog.cancel()

    # The multi_device leg (N > 1, or --multi-devices): a child process that
    # opens every device itself, started by rank 0 once all ranks have freed
    # their buffers and met; meanwhile the other ranks wait on the host
    # (host_side_wait), so no rank's collective kernel spins on a GPU the child
    # is timing.
    multi = None if bad else multi_device_list(args, world, ndev)
    if multi is not None:
        del sets, scratch, d_bm, d_status, events
        if devname == "cuda":
            cuda.synchronize()
            torch.cuda.empty_cache()
        if use_dist:
            dist.barrier()  # every rank's GPU work is done and its buffers freed
        if rank == 0:
            with markers.region("bench:multi_device"):
                try:
                    out["multi_device"] = run_multi_device_leg(args, multi, k, m, bs, S_per)
                except Exception as e:  # noqa: BLE001 - the field, never the line or the wait
                    out["multi_device"] = {"error": repr(e)[:200], "devices": multi}
        if use_dist:
            host_side_wait(dist, rank, "xec_bench_multi_device_done", args.multi_timeout + 600)
    if out is not None:
        print(json.dumps(out), file=result_out, flush=True)
    if use_dist:
        # The line is out; a teardown that never returns (a peer gone from a
        # collective) must not hold the run: the process leaves after 120 s.
        import threading
        teardown = threading.Timer(120.0, lambda: (print(
            f"rank {rank}: process-group teardown still running after 120 s; leaving",
            file=sys.stderr, flush=True), os._exit(1 if bad else 0)))
        teardown.daemon = True
        teardown.start()
        # the other ranks wait here while rank 0 writes its line, so nothing they
        # log while tearing down can land inside it when stdout and stderr share
        # one pipe
        dist.barrier()
        dist.destroy_process_group()
    if bad:
        sys.exit("verification failed")


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


if __name__ == "__main__":
    main()
