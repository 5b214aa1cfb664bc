"""Per-kernel code-object metadata of one or two libmcc.so builds (CPU only):
    python3 tools/co_meta.py libA.so [libB.so] [kernel-substring]
prints LDS (group segment), VGPR/AGPR/SGPR counts and scratch per kernel, side by side."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
KEYS = ("group_segment_fixed_size", "vgpr_count", "agpr_count", "sgpr_count", "private_segment_fixed_size")


def meta(lib):
    tmp = tempfile.mkdtemp()
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(tmp, "x.so")],
                   check=True, capture_output=True)
    blob = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
    out = {}
    for k, s in enumerate(starts):
        part = os.path.join(tmp, f"b{k}.bin")
        open(part, "wb").write(blob[s:starts[k + 1] if k + 1 < len(starts) else len(blob)])
        co = os.path.join(tmp, f"co{k}.o")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode or not os.path.getsize(co):
            continue
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
        # a kernel's keys are listed alphabetically around its .name: the ones before it ("- .agpr_count"
        # opens the entry) are held until the name is seen
        cur, pend = None, {}
        for line in notes.splitlines():
            if re.match(r"\s+- \.", line):
                cur, pend = None, {}
            m = re.match(r"\s+\.name:\s+(\S+)", line)
            if m and m.group(1).startswith("_Z"):
                cur = out.setdefault(m.group(1), {})
                cur.update(pend)
                continue
            m = re.match(r"\s+-?\s*\.(%s):\s+(\S+)" % "|".join(KEYS), line)
            if m:
                (cur if cur is not None else pend)[m.group(1)] = m.group(2)
    return out


args = sys.argv[1:]
pat = args.pop() if len(args) > 1 and not args[-1].endswith(".so") else None
ms = [meta(a) for a in args]
for name in sorted(set().union(*ms)):
    if pat and pat not in name:
        continue
    row = ["/".join(m.get(name, {}).get(k, "-") for k in KEYS) for m in ms]
    flag = "" if len(set(row)) == 1 else "  *"
    print(f"{name[:70]:70s} " + "  ".join(row) + flag)
