#!/usr/bin/env python3
"""Register / scratch report of the engine's gfx950 kernels (runs on the CPU: hipcc only).

For every kernel of the given .hip files: VGPRs, AGPRs, SGPRs, scratch bytes per lane, VGPR and
SGPR spills, occupancy and static LDS (hipcc -Rpass-analysis=kernel-resource-usage).  For the
kernels named with --map, the scratch (spill / reload) instructions of the device assembly are
mapped to the source line they belong to (-gline-tables-only), so a reader can see whether the
spills sit in hot loops or at batch boundaries.

    python3 tools/resource_report.py [--map sssp_batch_kernelILi8] > profiles/r04_resource_usage.md
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "shadow_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
         "-Wno-unused-result"]
FIELDS = ("TotalSGPRs", "VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
          "SGPRs Spill", "VGPRs Spill", "LDS Size [bytes/block]")


def remarks(src, defines):
    cmd = ["/opt/rocm/bin/hipcc"] + FLAGS + defines + [
        "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", os.devnull]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    kernels, cur = collections.OrderedDict(), None
    for line in out.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            kernels[cur] = {}
            continue
        m = re.search(r"remark:\s+([^:]+): (\S+) \[-Rpass", line)
        if m and cur is not None and m.group(1).strip() in FIELDS:
            kernels[cur][m.group(1).strip()] = m.group(2)
    return kernels


def scratch_map(src, defines, pattern):
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + defines +
                       ["-gline-tables-only", "--cuda-device-only", "-S", src, "-o", asm],
                       check=True, capture_output=True)
        text = open(asm).read().split("\n")
    files = {}
    for l in text:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[m.group(1)] = os.path.basename(m.group(3) or m.group(2))
    out = {}
    start = None
    for i, l in enumerate(text):
        if re.match(r"^_Z\S*%s\S*:" % pattern, l):
            start = i
            name = l.split(":")[0]
            end = i
            while not text[end].startswith(".Lfunc_end"):
                end += 1
            cur = "?"
            n = 0
            per = collections.Counter()
            for t in text[start:end]:
                m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", t)
                if m:
                    cur = "%s:%s" % (files.get(m.group(1), m.group(1)), m.group(2))
                    continue
                s = t.strip()
                if not s or s.startswith((".", ";")) or s.endswith(":"):
                    continue
                n += 1
                if "scratch_" in s:
                    per[(cur, s.split()[0])] += 1
            out[name] = (n, per)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", nargs="*", default=["topo_sssp_batch.hip", "topo_replay.hip",
                                                    "topo_kernels.hip"])
    ap.add_argument("--map", action="append", default=[], help="kernel name pattern to map")
    ap.add_argument("-D", action="append", default=[], help="extra define")
    a = ap.parse_args()
    defines = ["-D" + d for d in a.D]
    print("# Kernel resources (hipcc -Rpass-analysis=kernel-resource-usage, gfx950%s)\n" %
          ("; " + " ".join(defines) if defines else ""))
    print("| kernel | VGPRs | AGPRs | SGPRs | scratch B/lane | VGPR spills | SGPR spills | "
          "waves/SIMD | static LDS B |")
    print("|---|---|---|---|---|---|---|---|---|")
    for f in a.files:
        for k, r in remarks(os.path.join(CSRC, f), defines).items():
            if "rocprim" in k or "hipcub" in k:
                continue
            print("| `%s` | %s | %s | %s | %s | %s | %s | %s | %s |" % (
                k, r.get("VGPRs"), r.get("AGPRs"), r.get("TotalSGPRs"),
                r.get("ScratchSize [bytes/lane]"), r.get("VGPRs Spill"), r.get("SGPRs Spill"),
                r.get("Occupancy [waves/SIMD]"), r.get("LDS Size [bytes/block]")))
    for pat in a.map:
        for f in a.files:
            for name, (n, per) in scratch_map(os.path.join(CSRC, f), defines, pat).items():
                tot = sum(per.values())
                print("\n## Scratch instructions of `%s` (%d of %d instructions)\n" % (name, tot, n))
                print("| source line | instruction | count |")
                print("|---|---|---|")
                for (loc, op), c in sorted(per.items()):
                    print("| %s | %s | %d |" % (loc, op, c))
    return 0


if __name__ == "__main__":
    sys.exit(main())
