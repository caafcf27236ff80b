#!/usr/bin/env python
"""Per-launch HBM traffic of the bench's watched kernels from rocprofv3 --pmc passes (scripts/gpu_pmc.sh).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE
tallies 128-B read requests at 64 B, i.e. reports half of the bytes of wide reads -> x2.  The result is keyed
by the labels bench.py uses for its roofline entries and written to profiles/pmc_traffic_<precision>.json,
which bench.py reads to fill `roofline.traffic`.

    python scripts/pmc_traffic.py fast
"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PREC = {"0": "fp32", "1": "bf16", "2": "bf16x3", "3": "bf16x2", "5": "fp16", "6": "fp16-rowscaled"}
MODE = {("false", "false"): "NT", ("false", "true"): "NN", ("true", "true"): "TN"}


CHAIN_ROLES = {  # (bwd, KS0, NT2, NL, KEEP) -> the role label bench.py's chain_work gives the same launch
    (False, 5, 9, 3, True): "sdf_fwd", (False, 5, 9, 3, False): "sdf_infer_fwd",
    (False, 20, 8, 3, True): "radiance_fwd", (True, 17, 3, 3, False): "sdf_bwd", (True, 16, 10, 3, False): "radiance_bwd",
    (False, 3, 8, 4, True): "bg_base_fwd", (False, 18, 4, 4, True): "bg_head_fwd", (False, 18, 8, 4, True): "bg_head_fwd",
    (True, 16, 2, 4, False): "bg_base_bwd", (True, 8, 9, 4, False): "bg_head_bwd", (True, 16, 9, 4, False): "bg_head_bwd",
    (False, 16, 1, 3, True): "head_fwd", (True, 1, 8, 3, False): "head_bwd",
}


def label(name, grid=0):
    m = re.search(r"gemm_tn_grouped_kernel<(\d), (true|false)>", name)
    if m:
        return f"mms_gemm_tn_grouped:{PREC[m.group(1)]}:TN_grouped"
    m = re.search(r"gemm_tn_wide_kernel<(\d), \d+>", name)
    if m:   # (prec 5: the mixed fp16 launch, mms_gemm_tn_wide16)
        return f"mms_gemm_tn_wide{'16' if m.group(1) == '5' else ''}:{PREC[m.group(1)]}:TN_grouped"
    m = re.search(r"gemm_kernel<(\d), (true|false), (true|false), (true|false)>", name)
    if m:
        return f"mms_gemm:{PREC[m.group(1)]}:{MODE.get((m.group(2), m.group(3)), '??')}"
    m = re.search(r"chain_kernel<(\d), (\d+), \d+, \d+, (\d+), (true|false), \d, \d, \d, \d, (true|false), (\d)(?:, \w+)?>",
                  name)
    if m:
        key = (m.group(4) == "true", int(m.group(2)), int(m.group(3)), int(m.group(6)), m.group(5) == "true")
        return f"mms_mlp_chain:{PREC[m.group(1)]}:{CHAIN_ROLES.get(key, 'other')}"
    if "hashgrid_bwd" in name:
        # hashgrid_bwd_walk_kernel<GROUP, ...>: the SDF batch walks 5 rows (centre + 4 taps) per thread
        return "mms_hashgrid_bwd_grouped:sdf_taps" if "walk_kernel<5" in name else "mms_hashgrid_bwd_grouped:radiance_or_bg"
    if "sdf_panel_fwd_kernel<5" in name:
        return "mms_sdf_panel_fwd:sdf_taps"
    if "sdf_panel_fwd_kernel<1, true>" in name:
        return "mms_sdf_panel_rays_fwd:sampler"
    if "sdf_panel_fwd_kernel<1" in name:
        return "mms_sdf_panel_fwd:sampler"
    if "rad_panel_fwd" in name:
        return "mms_rad_panel_fwd:radiance"
    if "hashgrid_fwd_kernel" in name:
        # thread per (point, level): the SDF [centre | 4 taps] batch is the launch with > 200k points
        return "mms_hashgrid_fwd_grouped:sdf_taps" if grid > 200000 * 16 else "mms_hashgrid_fwd_grouped:other"
    return None


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        lab = label(r["Kernel_Name"], int(float(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)))
        if lab:
            acc[lab].append(float(r["Counter_Value"]) * 1024.0)
    return acc


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fast"
    base = os.path.join(ROOT, "gpurun_out")
    fetch = per_kernel(os.path.join(base, f"pmc_{prec}_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(base, f"pmc_{prec}_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    out = {"precision": prec, "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
           "bench.py --steps 5 --warmup 2; FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B)", "kernels": {}}
    for lab in sorted(set(fetch) | set(write)):
        f = fetch.get(lab, [])
        w = write.get(lab, [])
        fb = 2.0 * sum(f) / max(1, len(f))
        wb = sum(w) / max(1, len(w))
        out["kernels"][lab] = {"launches": len(f), "fetch_bytes_per_launch": round(fb), "write_bytes_per_launch":
                               round(wb), "hbm_bytes_per_launch": round(fb + wb)}
    dst = os.path.join(ROOT, "profiles", f"pmc_traffic_{prec}.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
