"""Kernel resources of the device code as the compiler reports them (-Rpass-analysis=
kernel-resource-usage): VGPRs, SGPRs, spilled SGPRs / VGPRs, scratch bytes per lane, waves per SIMD.
Compiles the instantiation units for the given stack classes and kernels.hip (device only), then
prints a markdown table.  Usage: python tools/resources.py [STK ...] > profiles/<round>/resources.md"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "--offload-arch=gfx950", "-Wall",
         "-Wno-unused-parameter", "-munsafe-fp-atomics", "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage"]


def remarks(src, defs):
    cmd = ["/opt/rocm/bin/hipcc", *FLAGS, *defs, "-c", os.path.join(ROOT, src), "-o", "/dev/null"]
    out = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT).stderr
    rows, cur = [], None
    for line in out.split("\n"):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark: +([A-Za-z \[\]/]+?): (\S+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    return rows


def demangle(n):
    d = subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    d = d.replace("lumo::dev::", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", d).replace("void ", "")


def main():
    stks = sys.argv[1:] or ["0", "4"]
    units = [(f"lumo_amd/csrc/device/inst_{k}.hip", [f"-DLUMO_STK={s}"]) for s in stks for k in ("pt", "bd")]
    units.append(("lumo_amd/csrc/device/kernels.hip", []))
    print("| kernel | VGPRs | SGPRs | SGPR spills | VGPR spills | scratch B/lane | waves/SIMD |")
    print("|---|---|---|---|---|---|---|")
    for src, defs in units:
        for r in remarks(src, defs):
            if "ScratchSize [bytes/lane]" not in r:
                continue
            print(f"| `{demangle(r['name'])}` | {r.get('VGPRs')} | {r.get('TotalSGPRs')} | {r.get('SGPRs Spill')} | "
                  f"{r.get('VGPRs Spill')} | {r.get('ScratchSize [bytes/lane]')} | {r.get('Occupancy [waves/SIMD]')} |")


if __name__ == "__main__":
    main()
