"""Register / occupancy report of the kernels TU for gfx950 (device-only -S, the product flags):
    python tools/kernel_regs.py [-DFOO ...] [--filter project_weight] [--keep out.s]
Prints NumVgprs, NumSgprs, scratch, occupancy and spill counts per kernel symbol."""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "slam-eslam_amd"))
import build_lib as B  # noqa: E402


def main():
    defs = [a for a in sys.argv[1:] if a.startswith("-D")]
    filt = "project_weight"
    keep = None
    extra = []
    args = sys.argv[1:]
    for i, a in enumerate(args):
        if a == "--filter":
            filt = args[i + 1]
        if a == "--keep":
            keep = args[i + 1]
        if a.startswith("-mllvm=") or a.startswith("-f"):
            extra.append(a)
    out = keep or tempfile.mktemp(suffix=".s")
    cmd = [B.HIPCC] + B.FLAGS + B.PER_SOURCE["eslam_kernels.hip"] + defs + extra + \
        ["--cuda-device-only", "-S", os.path.join(B.CSRC, "eslam_kernels.hip"), "-o", out]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    lines = open(out).read().split("\n")
    name = None
    info = {}
    for ln in lines:
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            name = m.group(1)
            info = {}
            continue
        m = re.match(r"^; (NumVgprs|NumSgprs|ScratchSize|Occupancy|LDSByteSize|NumVGPRsForWavesPerEU)[:\s]+(\S+)", ln.strip())
        if m and name:
            info[m.group(1)] = m.group(2)
            if m.group(1) == "Occupancy" and filt in name:
                print(f"{name[:90]:90s} vgpr={info.get('NumVgprs')} sgpr={info.get('NumSgprs')} "
                      f"scratch={info.get('ScratchSize')} occ={info.get('Occupancy')}")
    if not keep:
        os.unlink(out)


if __name__ == "__main__":
    main()
