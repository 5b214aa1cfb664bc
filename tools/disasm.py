"""Disassemble the gfx950 code object of a built libmcc.so (CPU only):
    python3 tools/disasm.py [lib.so] [out.s] [kernel-substring]
writes the whole listing to out.s (default /tmp/mcc.s) and prints the line ranges of the kernels whose
mangled name contains the substring."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
lib = sys.argv[1] if len(sys.argv) > 1 else "multi_camera_calibration_amd/libmcc.so"
out = sys.argv[2] if len(sys.argv) > 2 else "/tmp/mcc.s"
pat = sys.argv[3] if len(sys.argv) > 3 else None
tmp = tempfile.mkdtemp()
fat = os.path.join(tmp, "fat.bin")
subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(tmp, "x.so")], check=True)
blob = open(fat, "rb").read()
starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
text = []
for k, s in enumerate(starts):
    part = os.path.join(tmp, f"b{k}.bin")
    open(part, "wb").write(blob[s:starts[k + 1] if k + 1 < len(starts) else len(blob)])
    co = os.path.join(tmp, f"co{k}.o")
    r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
    if r.returncode or not os.path.getsize(co):
        continue
    text.append(subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                               capture_output=True, text=True).stdout)
open(out, "w").write("\n".join(text))
if pat:
    lines = open(out).read().splitlines()
    heads = [(i, l) for i, l in enumerate(lines) if re.match(r"^[0-9a-f]+ <.*>:$", l)]
    for j, (i, l) in enumerate(heads):
        if pat in l:
            end = heads[j + 1][0] if j + 1 < len(heads) else len(lines)
            print(i + 1, end, l)
