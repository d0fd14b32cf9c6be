#!/usr/bin/env python3
"""Turn one final tree's GPU passes into the files bench.py reads (run on the CPU host after
the passes' gpurun_out/ came back):

    python tools/pmc_finalize.py <tag>

* profiles/pmc_<tag>_<workload>.json for every workload whose PMC passes exist
  (gpurun_out/pmc_<tag>_<workload>_{rd,wr,dram,valu}/, tools/pmc_passes.sh), summarised by
  tools/pmc_summary.py with the workload's batch, or copied from gpurun_out/pmcsum/ where the
  box summarised them (tools/gpu_round.sh pmcsum);
* profiles/pmc_traffic.json: the north-star include? kernel's HBM bytes per launch (the
  line's roofline.traffic), with its source;
* profiles/rocprof_means.json from profiles/<tag>_kernel_stats.csv (tools/rocprof_means.py).

bench.PMC_FILES must then name the same tag (tests/test_profiles_tagged.py checks it)."""
import glob
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PASSES = ("rd", "wr", "dram", "valu", "stall", "fs", "ws")   # tools/pmc_passes.sh
BATCH = {"nstar": 1 << 24, "1m": 1 << 20, "1m_big": 1 << 24, "100m": 1 << 24, "10b": 1 << 24, "200b": 1 << 24,
         "lua_1m": 1 << 20, "model_P8_nstar": 1 << 24, "model_P8_200b": 1 << 24, "model_repl8_10b": 1 << 24}


def main():
    tag = sys.argv[1]
    # --box: run on the GPU box itself (tools/gpu_round.sh pmcsum): the summaries go to
    # gpurun_out/pmcsum/ and the raw counter CSVs are deleted, since a call's gpurun_out/ comes
    # back only below 64 MiB (the per-rank models' passes hold every torch kernel's rows too)
    box = "--box" in sys.argv[2:]
    outdir = os.path.join(ROOT, "gpurun_out", "pmcsum") if box else os.path.join(ROOT, "profiles")
    os.makedirs(outdir, exist_ok=True)
    for wl, batch in BATCH.items():
        # exactly this workload's passes ("1m_*" would also take "1m_big_*")
        dirs = [os.path.join(ROOT, "gpurun_out", "pmc_%s_%s_%s" % (tag, wl, p)) for p in PASSES]
        dirs = [d for d in dirs if os.path.isdir(d)]
        out = os.path.join(outdir, "pmc_%s_%s.json" % (tag, wl))
        made = os.path.join(ROOT, "gpurun_out", "pmcsum", "pmc_%s_%s.json" % (tag, wl))
        if dirs:
            subprocess.check_call([sys.executable, os.path.join(HERE, "pmc_summary.py"), *dirs, "--workload", wl,
                                   "--batch", str(batch), "--json", out], stdout=subprocess.DEVNULL)
        elif not box and os.path.exists(made):   # summarised on the box (pmcsum): take it as is
            shutil.copyfile(made, out)
        else:
            continue
        print("wrote", os.path.relpath(out, ROOT))
        if box:
            for d in dirs:
                shutil.rmtree(d)
            continue
        if wl == "nstar":
            rec = json.load(open(out))["nstar"]
            k = rec.get("bf_include_hash_kernel") or {}
            traffic = {"nstar": dict(rec, include_hash_kernel=k),   # (bench.py's kernel name for it)
                       "source": "profiles/pmc_%s_nstar.json" % tag}
            with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as fh:
                json.dump(traffic, fh, indent=1, sort_keys=True)
                fh.write("\n")
            print("wrote profiles/pmc_traffic.json")
    stats = os.path.join(ROOT, "profiles", "%s_kernel_stats.csv" % tag)
    if not box and os.path.exists(stats):
        txt = subprocess.check_output([sys.executable, os.path.join(HERE, "rocprof_means.py"),
                                       os.path.relpath(stats, ROOT), "--workload", "nstar"], cwd=ROOT, text=True)
        with open(os.path.join(ROOT, "profiles", "rocprof_means.json"), "w") as fh:
            fh.write(txt)
        print("wrote profiles/rocprof_means.json")


if __name__ == "__main__":
    main()
