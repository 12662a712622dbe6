"""Summarise a tools/profile_bench.sh run into profiles/<tag>_summary.md and the per-launch HBM
traffic JSONs bench.py reads for its roofline fields (keyed by the workload and the source hash
the bench line printed, so a summary never prices other code).

usage: python tools/summarize_prof.py gpurun_out/prof_r03 r03
"""
import csv
import glob
import json
import os
import sys

src, tag = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
outdir = os.path.join(ROOT, "profiles")
os.makedirs(outdir, exist_ok=True)


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0].replace("shdtopo::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0]


lines = ["# rocprofv3 summary %s (bench.py, 1 x MI355X)" % tag, ""]
stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
kavg = {}
if stats:
    lines += ["## kernel-trace --stats", "", "| kernel | calls | total ms | avg ms | % |",
              "|---|---|---|---|---|"]
    for r in csv.DictReader(open(stats[0])):
        lines.append("| %s | %s | %.3f | %.3f | %.2f |" % (
            short(r["Name"]), r["Calls"], float(r["TotalDurationNs"]) / 1e6,
            float(r["AverageNs"]) / 1e6, float(r["Percentage"])))
        kavg[short(r["Name"]).split("<")[0]] = float(r["AverageNs"]) / 1e6
    lines.append("")
per = {}
dur = {}
for f in glob.glob(os.path.join(src, "*", "*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"]).split("<")[0]
        per.setdefault(k, {})
        c = r["Counter_Name"]
        per[k][c] = per[k].get(c, 0.0) + float(r["Counter_Value"])
        dur.setdefault(k, {}).setdefault(c, set()).add(r.get("Dispatch_Id"))
lines += ["## PMC (summed over the kernel's dispatches, one pass per counter group)", ""]
for k, d in sorted(per.items()):
    if not any(x in k for x in ("sssp", "packet", "pair", "replay")):
        continue
    lines.append("### %s" % k)
    for c, v in sorted(d.items()):
        lines.append("* %s = %.6g (%d dispatches)" % (c, v, len(dur[k][c])))
    lines.append("")

# the bench line of the trace pass: its pmc keys name the workload and the code
bench = None
log = os.path.join(src, "trace.log")
if os.path.exists(log):
    for line in open(log).read().splitlines():
        if line.startswith("{"):
            bench = json.loads(line)


def per_launch(k, c):
    d = per.get(k, {})
    n = max(1, len(dur.get(k, {}).get(c, ())))
    return d.get(c, 0.0) / n


def traffic(k, key, extra=None):
    # gfx950 FETCH_SIZE / WRITE_SIZE are in KiB; random 64-B requests count at their size (the
    # kernels here issue no wide streaming reads that the counter would halve)
    fetch = per_launch(k, "FETCH_SIZE") * 1024
    write = per_launch(k, "WRITE_SIZE") * 1024
    rd = per_launch(k, "TCC_EA0_RDREQ_sum")
    wr = per_launch(k, "TCC_EA0_WRREQ_sum")
    at = per_launch(k, "TCC_EA0_ATOMIC_sum")
    out = dict(config_key=key, kernel=k, hbm_bytes_per_launch=fetch + write,
               dram_requests_per_launch=rd + wr, fetch_bytes=fetch, write_bytes=write,
               rdreq=rd, wrreq=wr, atomic_req=at, kernel_avg_ms_rocprof=kavg.get(k),
               source="rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_EA0_* (separate passes), "
                      "profiles/%s_summary.md" % tag)
    if extra:
        out.update(extra)
    return out


def emit(name, obj, k):
    json.dump(obj, open(os.path.join(outdir, "%s_%s_pmc.json" % (tag, name)), "w"), indent=1)
    lines.extend(["## per-launch HBM traffic of %s" % k, "",
                  "* FETCH_SIZE %.4g B + WRITE_SIZE %.4g B = %.4g B per launch" %
                  (obj["fetch_bytes"], obj["write_bytes"], obj["hbm_bytes_per_launch"]),
                  "* DRAM read requests %.4g, write requests %.4g, atomics %.4g per launch" %
                  (obj["rdreq"], obj["wrreq"], obj["atomic_req"]),
                  "* rocprofv3 average duration %s ms" % obj["kernel_avg_ms_rocprof"], ""])
    if obj["kernel_avg_ms_rocprof"]:
        t = obj["kernel_avg_ms_rocprof"] / 1e3
        lines.append("* measured %.1f GB/s = %.3f of the 8 TB/s HBM peak; %.3g DRAM requests/s" % (
            obj["hbm_bytes_per_launch"] / t / 1e9, obj["hbm_bytes_per_launch"] / t / 8e12,
            obj["dram_requests_per_launch"] / t))
        lines.append("")


if bench:
    key = bench["roofline"]["pmc_key"]
    if "sssp_batch_kernel" in per:
        emit("sssp", traffic("sssp_batch_kernel", key + "-sssp_batch_kernel"),
             "sssp_batch_kernel")
    if "heap_replay_kernel" in per and bench["sssp"].get("tie_dense"):
        rp = bench.get("replay", {})
        extra = {}
        if rp.get("pops"):
            rows = bench["roofline"]["units_per_launch"]
            # pops per launch of the timed build (every row replayed)
            extra["pops_per_launch"] = rp["pops"]
        emit("replay", traffic("heap_replay_kernel", key + "-heap_replay_kernel", extra),
             "heap_replay_kernel")
        obj = json.load(open(os.path.join(outdir, "%s_replay_pmc.json" % tag)))
        if obj.get("pops_per_launch"):
            obj["lines_per_pop"] = round((obj["rdreq"] + obj["wrreq"]) / obj["pops_per_launch"], 2)
            json.dump(obj, open(os.path.join(outdir, "%s_replay_pmc.json" % tag), "w"), indent=1)
    rr = bench.get("route_roofline") or {}
    if "packet_route_kernel" in per and rr.get("pmc_key"):
        emit("route", traffic("packet_route_kernel", rr["pmc_key"]), "packet_route_kernel")
open(os.path.join(outdir, "%s_summary.md" % tag), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
