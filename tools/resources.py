"""Per-kernel resource usage of the shipped library (VGPRs, AGPRs, SGPRs, spills, scratch
bytes per lane, LDS bytes per workgroup, occupancy in waves per SIMD), from the gfx950 code
generator's kernel-resource-usage remarks for each source the Makefile links into
libnarwhal_amd.so, with the Makefile's flags. Prints a fixed-width table (committed as
profiles/r04*/resources.txt). Runs on the CPU; build tooling, not product code."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ["nw_kernels.hip", "nw_batch.hip", "nw_cert.hip", "nw_small.hip"]
FIELDS = [("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("TotalSGPRs", "sgpr"),
          ("VGPRs Spill", "vspill"), ("SGPRs Spill", "sspill"),
          ("ScratchSize [bytes/lane]", "scratch"), ("LDS Size [bytes/block]", "lds"),
          ("Occupancy [waves/SIMD]", "occ")]


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names),
                             capture_output=True, text=True, check=True).stdout.split("\n")
        return out[:len(names)]
    except (OSError, subprocess.CalledProcessError):
        return names


def remarks(src, extra):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "narwhal_amd/csrc"),
           "-Wno-unused-function", "-x", "hip", "-c", src, "-o", os.devnull,
           "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage"] + extra
    err = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\S+) \[-Rpass", line)
        if m and cur is not None:
            for key, short in FIELDS:
                if m.group(1).strip() == key:
                    cur[short] = m.group(2)
    return rows


def main():
    extra = sys.argv[1:]
    print(f"# gfx950 kernel resources, hipcc -O3 {' '.join(extra)}".rstrip())
    print(f"{'kernel':58s} {'vgpr':>5s} {'agpr':>5s} {'sgpr':>5s} {'vspill':>6s} "
          f"{'sspill':>6s} {'scratch':>7s} {'lds':>6s} {'occ':>4s}  source")
    for src in SOURCES:
        rows = remarks(os.path.join(ROOT, "narwhal_amd/csrc", src), extra)
        names = demangle([r["name"] for r in rows])
        for r, nm in zip(rows, names):
            nm = nm.replace("nw::", "").replace("(anonymous namespace)::", "")
            nm = nm.split("(")[0].removeprefix("void ")
            nm = nm if len(nm) <= 58 else nm[:55] + "..."
            print(f"{nm:58s} {r.get('vgpr', '?'):>5s} {r.get('agpr', '?'):>5s} "
                  f"{r.get('sgpr', '?'):>5s} {r.get('vspill', '?'):>6s} {r.get('sspill', '?'):>6s} "
                  f"{r.get('scratch', '?'):>7s} {r.get('lds', '?'):>6s} {r.get('occ', '?'):>4s}  {src}")


if __name__ == "__main__":
    main()
