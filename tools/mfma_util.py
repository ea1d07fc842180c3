#!/usr/bin/env python3
"""MFMA utilisation per kernel / 3x3x3 conv shape from one rocprofv3 PMC pass over a bench step.

    rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
        -d gpurun_out/pmc_mfma -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 ...
    python3 tools/mfma_util.py gpurun_out/pmc_mfma [--md out.md]

Per (kernel, grid) group, averaged over its launches (counter rows summed over XCD / SE
instances first):
  * flops    = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 (one MOP = 512 bf16 FLOPs)
  * busy     = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1,024 SIMDs): the fraction of
               the chip's SIMD-cycles spent issuing matrix instructions during the kernel
  * tflops   = flops / kernel duration (profiled timestamps), frac of the 2.5 PF dense bf16 peak
  * ceiling  = min(1, AI x 8 TB/s / 2.5 PF) for the 3x3x3 shapes below, AI = the shape's useful
               FLOPs / algorithmic HBM bytes: the utilisation an HBM-bound
               kernel of that shape can reach at all
  * useful / ceiling = (useful TFLOP/s / 2.5 PF) / ceiling: how far the kernel is from its shape's
               roofline, in matrix-core terms
"""
import collections
import csv
import glob
import re
import sys

PEAK_TF = 2500.0
HBM_TBS = 8.0

# useful FLOPs and algorithmic bytes per launch of the 3x3x3 engines at the headline config (3-layer
# published, 512^2 x 128, bf16); vox = voxels of the grid the kernel runs on
_V128 = 128 * 128 * 32
_V512 = 512 * 512 * 128
_V256 = 256 * 256 * 64
_V32 = 32 * 32 * 8
SHAPES = [
    # (kernel regex, production grid in WORKGROUPS (r05 step trace), shape, useful flops, algorithmic
    # bytes).  A kernel is attributed to a shape only at that shape's production grid: the same
    # template also runs on other grids (e.g. k_col_bwd<4, 2> on a 64^2 x 16 level) whose useful
    # work is different, and those rows get no shape columns.
    (r"k_pm_fwd", 768, "18-ch block fwd (chained): 3x3x3 9->9 + 1x1 9->18 + next 1x1 18->9 @128^2x32",
     2 * _V128 * (2187 + 162 + 162), _V128 * 63 * 2),
    (r"k_pm_bwd2", 256, "18-ch block dgrad (chained): 3x3x3 9->9 + 1x1 9->18 + previous 1x1 18->9 @128^2x32",
     2 * _V128 * (2187 + 162 + 162), _V128 * 99 * 2),
    (r"k_pm_w2grad<32>", 256, "18-ch block wgrad: 3x3x3 9->9 @128^2x32", 2 * _V128 * 2187, _V128 * 18 * 2),
    (r"k_pm_w2grad<64>", 2048, "up-block conv2 wgrad: 3x3x3 9->9 @256^2x64", 2 * _V256 * 2187, _V256 * 18 * 2),
    (r"k_wide_fwd", 256, "72-ch block fwd: 3x3x3 36->36 + 2x 1x1 @32^2x8", 2 * _V32 * (34992 + 5184),
     _V32 * (144 * 4 + 72 * 2)),
    (r"k_wide_bwd_data", 256, "72-ch block dgrad: 3x3x3 36->36 + 2x 1x1 @32^2x8", 2 * _V32 * (34992 + 5184),
     _V32 * (216 * 4 + 72 * 2)),
    (r"k_wide_wgrad", 208, "72-ch block wgrad: 3x3x3 36->36 + 2x 1x1 @32^2x8", 2 * _V32 * (34992 + 5184),
     _V32 * (144 * 4 + 72 * 2)),
    (r"k_col_fwd<4, 2[,>]", 2048, "4-ch block fwd: 3x3x3 2->2 @512^2x128", 2 * _V512 * (108 + 16), _V512 * 12 * 2),
    (r"k_col_bwd<4, 2[,>]", 2048, "4-ch block bwd: 3x3x3 2->2 dgrad + wgrad @512^2x128", 4 * _V512 * (108 + 16),
     _V512 * 16 * 2),
    (r"k_col_fwd<8, 4[,>]", 512, "8-ch block fwd: 3x3x3 4->4 @256^2x64", 2 * _V256 * (432 + 64), _V256 * 24 * 2),
    (r"k_col_bwd<8, 4[,>]", 512, "8-ch block bwd: 3x3x3 4->4 dgrad + wgrad @256^2x64", 4 * _V256 * (432 + 64),
     _V256 * 32 * 2),
    (r"k_col_fwd<2, 1[,>]", 512, "2-ch block fwd: 3x3x3 1->1 @128^2x32", 2 * _V128 * (27 + 4), _V128 * 6 * 2),
    (r"k_col_bwd<2, 1[,>]", 512, "2-ch block bwd: 3x3x3 1->1 @128^2x32", 4 * _V128 * (27 + 4), _V128 * 8 * 2),
    (r"k_lines<1, 8, false>", 1024, "up-block conv2 fwd: 3x3x3 4->4 @512^2x128", 2 * _V512 * 432, _V512 * 8 * 2),
    (r"k_lines<1, 8, true>", 1024, "up-block conv2 dgrad: 3x3x3 4->4 @512^2x128", 2 * _V512 * 432, _V512 * 8 * 2),
    (r"k_wgrad_ds<4, 4, 3, 1, 1,", 512, "up-block conv2 wgrad (D-shifted MFMA): 3x3x3 4->4 @512^2x128",
     2 * _V512 * 432, _V512 * 8 * 2),
]


def shape_of(name, grid):
    for pat, g, desc, fl, by in SHAPES:
        if re.search(pat, name) and grid == g:
            return desc, fl, by
    return None


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("vq3d::", "")
    n = re.sub(r"^void ", "", n)
    return re.sub(r"\(.*$", "", n)


def main():
    d = sys.argv[1]
    md = sys.argv[sys.argv.index("--md") + 1] if "--md" in sys.argv else None
    vals = collections.defaultdict(float)
    meta = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "vq3d" not in r["Kernel_Name"]:
                continue
            key = (f, r["Dispatch_Id"])
            wg = int(r.get("Workgroup_Size") or r.get("Workgroup_Size_X") or 1)
            meta[key] = (short(r["Kernel_Name"]), int(r["Grid_Size"]) // max(wg, 1),
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
            vals[(key, r["Counter_Name"])] += float(r["Counter_Value"])
    groups = collections.defaultdict(list)
    for key, (name, grid, us) in meta.items():
        groups[(name, grid)].append((us, vals[(key, "SQ_INSTS_VALU_MFMA_MOPS_BF16")],
                                     vals[(key, "SQ_VALU_MFMA_BUSY_CYCLES")], vals[(key, "GRBM_GUI_ACTIVE")]))
    rows = []
    for (name, grid), ls in groups.items():
        n = len(ls)
        us = sum(x[0] for x in ls) / n
        mops = sum(x[1] for x in ls) / n
        busy = sum(x[2] for x in ls) / n
        grbm = sum(x[3] for x in ls) / n
        if mops == 0:
            continue
        flops = mops * 512
        tf = flops / (us * 1e-6) / 1e12
        util = busy / (grbm / 8 * 1024) if grbm else 0.0
        sh = shape_of(name, grid)
        ceil = useful_tf = None
        if sh:
            ai = sh[1] / sh[2]
            ceil = min(1.0, ai * HBM_TBS * 1e12 / (PEAK_TF * 1e12))
            useful_tf = sh[1] / (us * 1e-6) / 1e12
            # the matrix cores cannot do less work than the shape's useful FLOPs: a shape whose
            # useful work exceeds what the kernel issued is a wrong attribution, so fail loudly
            if sh[1] > flops * 1.0001:
                raise SystemExit(f"{name} [{grid}]: useful {sh[1]:.3e} FLOPs > issued {flops:.3e}: wrong shape")
        rows.append((n * us, name, grid, n, us, flops, tf, util, sh, ceil, useful_tf))
    rows.sort(reverse=True)
    out = ["| kernel [workgroups] | launches | avg us (profiled) | shape | MFMA GFLOP/launch (MOPS x 512) | "
           "TFLOP/s | frac of 2.5 PF | MFMA busy (counter) | useful TFLOP/s | shape ceiling min(1, AI*8TB/s/2.5PF) | "
           "useful / ceiling |",
           "|---|---|---|---|---|---|---|---|---|---|---|"]
    for tot, name, grid, n, us, flops, tf, util, sh, ceil, utf in rows:
        out.append(f"| `{name}` [{grid}] | {n} | {us:.1f} | {sh[0] if sh else ''} | {flops / 1e9:.3f} | {tf:.1f} | "
                   f"{tf / PEAK_TF:.4f} | {util:.4f} | {'' if utf is None else f'{utf:.1f}'} | "
                   f"{'' if ceil is None else f'{ceil:.3f}'} | "
                   f"{'' if ceil is None else f'{utf / PEAK_TF / ceil:.3f}'} |")
    text = "\n".join(out)
    print(text)
    if md:
        open(md, "w").write(text + "\n")


if __name__ == "__main__":
    main()
