"""Per-kernel register / scratch / occupancy report of the gfx950 kernels, from the compiler
(`-Rpass-analysis=kernel-resource-usage`, device-only compiles with the build's own flags).

    python scripts/kernel_resources.py [file.hip ...] [--filter SUBSTR] [-j N]

Prints one row per kernel instance: VGPRs, AGPRs, SGPR spills, VGPR spills, scratch bytes per
lane, LDS bytes, occupancy (waves/SIMD).  Exit status 1 if any kernel needs scratch (a private
copy of a by-value argument or spilled registers in memory: tests/test_kernel_resources.py)."""
import argparse
import concurrent.futures as cf
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, "cori_intml_examples_amd", "csrc", "kernels")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-I" + KDIR, "-munsafe-fp-atomics",
         "-mllvm", "-amdgpu-mfma-vgpr-form", "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage"]
FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill",
          "ScratchSize [bytes/lane]": "scratch", "LDS Size [bytes/block]": "lds", "Occupancy [waves/SIMD]": "occ"}


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), text=True,
                             capture_output=True, timeout=60).stdout.splitlines()
        return out if len(out) == len(names) else names
    except Exception:              # noqa: BLE001
        return names


def report(src):
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    r = subprocess.run([hipcc] + FLAGS + ["-c", src, "-o", os.devnull], capture_output=True, text=True, timeout=1800)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1), "file": os.path.basename(src)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s+(-?\d+)", line)
        if m and cur is not None and m.group(1).strip() in FIELDS:
            cur[FIELDS[m.group(1).strip()]] = int(m.group(2))
    if r.returncode != 0:
        raise RuntimeError("%s: %s" % (src, r.stderr[-2000:]))
    return [x for x in rows if "vgpr" in x]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="*")
    ap.add_argument("--filter", default="")
    ap.add_argument("-j", type=int, default=4)
    args = ap.parse_args()
    files = args.files or sorted(os.path.join(KDIR, f) for f in os.listdir(KDIR) if f.endswith(".hip"))
    rows = []
    with cf.ThreadPoolExecutor(args.j) as ex:
        for rs in ex.map(report, files):
            rows += rs
    names = demangle([r["name"] for r in rows])
    bad = 0
    print("%-6s %-5s %-6s %-6s %-7s %-6s %-4s  %s" % ("VGPR", "AGPR", "SSpill", "VSpill", "scratch", "LDS", "occ", "kernel (file)"))
    for r, n in zip(rows, names):
        if args.filter and args.filter not in n:
            continue
        bad += r.get("scratch", 0) > 0
        print("%-6d %-5d %-6d %-6d %-7d %-6d %-4d  %s (%s)" % (r["vgpr"], r.get("agpr", 0), r.get("sgpr_spill", 0),
                                                           r.get("vgpr_spill", 0), r.get("scratch", 0), r.get("lds", 0),
                                                           r.get("occ", 0), n[:150], r["file"]))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
