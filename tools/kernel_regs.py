"""Register counts and spills of the kernels in a built libmhppo.so (code-object metadata notes).

usage: python tools/kernel_regs.py [libmhppo.so] [name-substring]"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import check_asm_rd  # noqa: E402

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def kernels(lib):
    for co in check_asm_rd.code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            out = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True).stdout
        for m in re.finditer(r"\.name:\s+(\S+).*?\.sgpr_spill_count:\s+(\d+).*?\.vgpr_count:\s+(\d+)"
                             r".*?\.vgpr_spill_count:\s+(\d+)", out, re.S):
            yield m.group(1), int(m.group(3)), int(m.group(4)), int(m.group(2))


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(check_asm_rd.ROOT, "mh-ppo_amd", "mhppo", "lib",
                                                             "libmhppo.so")
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, v, vs, ss in kernels(lib):
        if sub in name:
            print(f"{name[:100]:100s} vgpr {v:3d} vgpr_spill {vs} sgpr_spill {ss}")
