"""rocprofv3 outputs under gpurun_out/ -> one markdown report for profiles/.

    python tools/profile_report.py <title> <out.md> [prof_dir] [pmc_dir] [out.json]

prof_dir: `--kernel-trace --stats --output-format csv -o run` output (kernel stats + trace);
pmc_dir:  tools/gpu_pmc.sh output (one sub-directory per counter pass).
Sections: per-kernel duration stats, the last step's kernel timeline (start/end relative to
that step's encoder launch, queue id), and per-launch PMC averages with HBM traffic
(FETCH_SIZE x 2, the gfx950 half-count correction of MI355X_MICROARCH.md, + WRITE_SIZE; KB).
out.json (optional): the per-kernel HBM bytes per launch that bench.py reports as roofline.traffic.
"""
import json
import collections
import csv
import os
import sys


def kernel_stats(prof):
    rows = list(csv.DictReader(open(os.path.join(prof, "run_kernel_stats.csv"))))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = ["| kernel | calls | avg us | min us | max us | total % |", "|---|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        out.append("| `%s` | %s | %.1f | %.1f | %.1f | %.1f |" % (
            r["Name"].split("(")[0][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3,
            float(r["MaxNs"]) / 1e3, 100.0 * float(r["TotalDurationNs"]) / tot))
    return out


def timeline(prof):
    rows = list(csv.DictReader(open(os.path.join(prof, "run_kernel_trace.csv"))))
    rows = [r for r in rows if r["Kernel_Name"].startswith("dad_")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("dad_encode")]
    if len(starts) < 2:
        return []
    a, b = starts[-2], starts[-1]
    base = int(rows[a]["Start_Timestamp"])
    out = ["| kernel | queue | start us | end us | dur us |", "|---|---|---|---|---|"]
    for r in rows[a:b + 1]:
        s, e = int(r["Start_Timestamp"]) - base, int(r["End_Timestamp"]) - base
        out.append("| `%s` | %s | %.1f | %.1f | %.1f |" % (r["Kernel_Name"].split("(")[0], r.get("Queue_Id", ""),
                                                           s / 1e3, e / 1e3, (e - s) / 1e3))
    out.append("")
    out.append("Step period (encoder start to next encoder start): %.1f us" % (
        (int(rows[b]["Start_Timestamp"]) - base) / 1e3))
    return out


def pmc_agg(pmc_dir):
    agg = collections.defaultdict(list)
    for name in sorted(os.listdir(pmc_dir)):
        f = os.path.join(pmc_dir, name, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


N_SIMDS = 1024   # MI355X: 256 CUs x 4 SIMDs


def lib_sha16():
    import hashlib
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                     "robust-speech-emotion-recognition-via-dynamic-asymmetric-distillation-in-noisy-environments_amd",
                     "lib", "libdad_hip.so")
    try:
        return hashlib.sha256(open(p, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def pmc_json(pmc_dir, title):
    agg = pmc_agg(pmc_dir)
    mean = lambda k, c: (sum(agg[(k, c)]) / len(agg[(k, c)])) if agg.get((k, c)) else None
    out = {}
    for k in sorted({k for k, _ in agg}):
        f, w = mean(k, "FETCH_SIZE"), mean(k, "WRITE_SIZE")
        e = {}
        if f is not None and w is not None:
            e.update({"hbm_bytes_per_launch": (2 * f + w) * 1024.0, "fetch_kb_x2": 2 * f, "write_kb": w,
                      "launches": len(agg[(k, "FETCH_SIZE")])})
        mb, ga = mean(k, "SQ_VALU_MFMA_BUSY_CYCLES"), mean(k, "GRBM_GUI_ACTIVE")
        if mb is not None and ga:
            # busy cycles summed over SIMDs / (SIMDs x kernel cycles); GRBM_GUI_ACTIVE sums 8 XCDs
            e["mfma_busy_frac"] = mb / (N_SIMDS * ga / 8.0)
            e["mfma_busy_cycles"] = mb
        if e:
            out[k] = e
    return {"source": title, "lib_sha16": lib_sha16(),
            "units": "bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) KB x 1024; mfma_busy_frac = "
                     "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)", "kernels": out}


def pmc(pmc_dir):
    agg = collections.defaultdict(list)
    for name in sorted(os.listdir(pmc_dir)):
        f = os.path.join(pmc_dir, name, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
    kernels = sorted({k for k, _ in agg})
    counters = sorted({c for _, c in agg})
    out = ["| kernel | " + " | ".join(counters) + " | HBM KB (2*FETCH+WRITE) |",
           "|---|" + "---|" * (len(counters) + 1)]
    for k in kernels:
        vals = {c: sum(agg[(k, c)]) / len(agg[(k, c)]) for c in counters if agg.get((k, c))}
        traffic = ""
        if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
            traffic = "%.0f" % (2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"])
        out.append("| `%s` | " % k + " | ".join("%.0f" % vals[c] if c in vals else "" for c in counters) +
                   " | %s |" % traffic)
    return out


def main():
    title, dst = sys.argv[1], sys.argv[2]
    prof = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/prof"
    pmc_dir = sys.argv[4] if len(sys.argv) > 4 else "gpurun_out/pmc"
    out = ["# " + title, ""]
    if os.path.isdir(prof):
        out += ["## Kernel durations (rocprofv3 --kernel-trace --stats)", ""] + kernel_stats(prof)
    tl = timeline(prof) if os.path.isdir(prof) else []
    if tl:
        out += ["", "## Last profiled step: kernel timeline", ""] + tl
    if os.path.isdir(pmc_dir):
        out += ["", "## PMC per launch (averages over launches; separate --pmc passes)", ""] + pmc(pmc_dir)
    open(dst, "w").write("\n".join(out) + "\n")
    if len(sys.argv) > 5 and os.path.isdir(pmc_dir):
        json.dump(pmc_json(pmc_dir, title), open(sys.argv[5], "w"), indent=1)


if __name__ == "__main__":
    main()
