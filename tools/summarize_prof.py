"""Summarise a tools/profile_bench.sh run into profiles/<tag>_summary.md and the per-launch HBM
traffic JSON bench.py reads for roofline.traffic.

usage: python tools/summarize_prof.py gpurun_out/prof_r01 r01
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
    n = name.split("(")[0].replace("shdtopo::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("<")[0] if n.startswith("sssp_rows_kernel") else n.split("(")[0]


lines = ["# rocprofv3 summary %s (bench.py, C4/C5, 1 x MI355X)" % tag, ""]
stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
if stats:
    lines += ["## kernel-trace --stats", "", "| kernel | calls | total ms | avg ms | % |",
              "|---|---|---|---|---|"]
    for r in csv.DictReader(open(stats[0])):
        lines.append("| %s | %s | %.3f | %.3f | %.2f |" % (
            short(r["Name"]), r["Calls"], float(r["TotalDurationNs"]) / 1e6,
            float(r["AverageNs"]) / 1e6, float(r["Percentage"])))
    lines.append("")
per = {}
dur = {}
for f in glob.glob(os.path.join(src, "*", "*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        per.setdefault(k, {})
        c = r["Counter_Name"]
        per[k][c] = per[k].get(c, 0.0) + float(r["Counter_Value"])
        disp = r.get("Dispatch_Id")
        dur.setdefault(k, set()).add(disp)
lines += ["## PMC (summed over the kernel's dispatches, one pass per group)", ""]
for k, d in sorted(per.items()):
    if "sssp" not in k and "packet" not in k and "pair" not in k:
        continue
    lines.append("### %s (%d dispatches)" % (k, len(dur[k])))
    for c, v in sorted(d.items()):
        lines.append("* %s = %.6g" % (c, v))
    lines.append("")
ks = [k for k in per if k.startswith("sssp_")]
if ks:
    k = ks[0]
    d = per[k]
    n = max(1, len(dur[k]))
    fetch = d.get("FETCH_SIZE", 0.0) * 1024 / n
    write = d.get("WRITE_SIZE", 0.0) * 1024 / n
    rd = d.get("TCC_EA0_RDREQ_sum", 0.0) / n
    wr = d.get("TCC_EA0_WRREQ_sum", 0.0) / n
    at = d.get("TCC_EA0_ATOMIC_sum", 0.0) / n
    # config key and the batch kernel's streaming sweep bytes as bench.py reports them (its JSON
    # line in the trace pass' log)
    log = open(os.path.join(src, "trace.log")).read() if os.path.exists(
        os.path.join(src, "trace.log")) else ""
    key = None
    sweep_bytes = 0
    for line in log.splitlines():
        if line.startswith("{"):
            j = json.loads(line)
            c = j["config"]
            key = "C4-%d-%d-%d-rows%d-%s" % (c["vertices"], c["edges"], c["sources"],
                                             j["roofline"]["units_per_launch"], k)
            sweep_bytes = j.get("sssp", {}).get("sweep_bytes", 0)
    # gfx950: FETCH_SIZE counts wide (16 B/lane) streaming reads at half -- the sweeps are such
    # reads, so their missing half is added back (MI355X_MICROARCH.md, HBM/rocprofv3 section)
    fetch_c = fetch + sweep_bytes / 2
    out = dict(config_key=key, kernel=k, hbm_bytes_per_launch=fetch_c + write,
               dram_requests_per_launch=rd + wr,
               fetch_bytes=fetch, fetch_bytes_corrected=fetch_c, sweep_bytes=sweep_bytes,
               write_bytes=write, rdreq=rd, wrreq=wr, atomic_req=at,
               source="rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), profiles/%s_summary.md; "
                      "FETCH_SIZE per the gfx950 formula (64-B random requests counted at 64 B)%s"
                      % (tag, ", plus half of the sweeps' streaming bytes (counted at 1/2 on gfx950)"
                         if sweep_bytes else "; no streaming correction (sweeps read pending "
                         "vertices' 64-B lines only)"))
    json.dump(out, open(os.path.join(outdir, "%s_sssp_pmc.json" % tag), "w"), indent=1)
    lines += ["## per-launch HBM traffic of %s" % k, "",
              "* FETCH_SIZE = %.4g B, + streaming-sweep correction %.4g B = %.4g B" %
              (fetch, sweep_bytes / 2, fetch_c),
              "* WRITE_SIZE = %.4g B" % write,
              "* HBM traffic per launch = %.4g B" % (fetch_c + write),
              "* read requests %.4g, write requests %.4g, atomic requests %.4g per launch" %
              (rd, wr, at), ""]
rk = [k for k in per if k.startswith("packet_route")]
if rk:
    k = rk[0]
    d = per[k]
    n = max(1, len(dur[k]))
    fetch = d.get("FETCH_SIZE", 0.0) * 1024 / n
    write = d.get("WRITE_SIZE", 0.0) * 1024 / n
    json.dump(dict(kernel=k, hbm_bytes_per_launch=fetch + write, fetch_bytes=fetch,
                   write_bytes=write, dispatches=n,
                   source="rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, profiles/%s_summary.md" % tag),
              open(os.path.join(outdir, "%s_route_pmc.json" % tag), "w"), indent=1)
    lines += ["## per-launch HBM traffic of %s" % k, "",
              "* FETCH_SIZE = %.4g B, WRITE_SIZE = %.4g B, total %.4g B per launch" %
              (fetch, write, fetch + write), ""]
open(os.path.join(outdir, "%s_summary.md" % tag), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
