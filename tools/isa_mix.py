#!/usr/bin/env python3
"""Static instruction mix of gfx950 kernels (CPU only): compiles a .hip source for the device,
disassembles it, and counts the instructions of every kernel whose symbol contains a pattern.

  python tools/isa_mix.py circulantpreconditioner_amd/csrc/cfp_three_pass.hip k_tp_mid_sw

Per kernel: total, f64 VALU, other VALU, cross-lane moves (DPP, permlane), LDS, global memory
and scalar instructions.  The counts are of the code, not of its execution (loops count once).
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

HIPCC = "/opt/rocm/bin/hipcc"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def categorize(op: str) -> str:
    if op.startswith("v_"):
        if "permlane" in op:
            return "permlane"
        if op.endswith("_dpp") or "_dpp" in op:
            return "dpp"
        if "f64" in op:
            return "valu_f64"
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main() -> int:
    src, pat = sys.argv[1], sys.argv[2]
    csrc = os.path.dirname(os.path.abspath(src))
    with tempfile.TemporaryDirectory() as td:
        obj = os.path.join(td, "dev.o")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--offload-device-only",
                        "--no-gpu-bundle-output", "-I", csrc, "-c", src, "-o", obj], check=True,
                       stderr=subprocess.DEVNULL)
        dis = subprocess.run([OBJDUMP, "-d", obj], check=True, capture_output=True, text=True).stdout
    kern, counts = None, {}
    for line in dis.split("\n"):
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            kern = m.group(1) if pat in m.group(1) else None
            if kern:
                counts[kern] = collections.Counter()
            continue
        if kern:
            m = re.match(r"\s+([a-z_0-9]+)", line)
            if m:
                counts[kern][categorize(m.group(1))] += 1
    for k, c in counts.items():
        tot = sum(c.values())
        print(f"{k}\n  total {tot}: " + ", ".join(f"{n} {c[n]}" for n in
              ("valu_f64", "valu_other", "dpp", "permlane", "lds", "vmem", "salu", "other")))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
