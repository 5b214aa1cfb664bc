"""The gfx950 code objects inside libmcc.so (CPU: read from the built library, no GPU).

Every kernel runs without a stack: no scratch (private segment 0), no dynamic stack, no VGPR spills.
A kernel that needs a stack -- an out-of-line device call is enough -- gets a scratch setup on every
launch; round 4 measured that at +5 us per config4 step and +6 us per config3 step (one
__noinline__ helper in k_schur), so it is a regression this test catches before a GPU run.  Also
checked: every kernel the host launches is present, and the k_group variants stay at <= 256 VGPRs (two
waves per SIMD for their 512-thread workgroups)."""
import os
import re
import subprocess

import pytest

from multi_camera_calibration_amd import api

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _kernels(tmp):
    lib = api.build()
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(tmp, "x.so")],
                   check=True, capture_output=True)
    blob = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
    kernels = {}
    for k, s in enumerate(starts):
        part = os.path.join(tmp, f"b{k}.bin")
        end = starts[k + 1] if k + 1 < len(starts) else len(blob)
        with open(part, "wb") as f:
            f.write(blob[s:end])
        co = os.path.join(tmp, f"co{k}.o")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode != 0 or not os.path.getsize(co):
            continue
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
        cur = None
        for line in notes.splitlines():
            m = re.match(r"\s+\.name:\s+(\S+)", line)
            if m and m.group(1).startswith("_Z"):
                cur = kernels.setdefault(m.group(1), {})
                continue
            m = re.match(r"\s+\.(private_segment_fixed_size|uses_dynamic_stack|vgpr_spill_count|vgpr_count):\s+(\S+)", line)
            if m and cur is not None:
                cur[m.group(1)] = m.group(2)
    return kernels


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    if not os.path.exists(f"{LLVM}/clang-offload-bundler"):
        pytest.skip("no ROCm LLVM tools")
    return _kernels(str(tmp_path_factory.mktemp("co")))


def test_every_kernel_runs_without_a_stack(kernels):
    assert len(kernels) > 50
    bad = {k: v for k, v in kernels.items()
           if v.get("private_segment_fixed_size") != "0" or v.get("uses_dynamic_stack") != "false"
           or v.get("vgpr_spill_count") != "0"}
    assert not bad, bad


def test_launched_kernels_present(kernels):
    names = " ".join(kernels)
    for k in ("k_linearize", "k_group", "k_prep", "k_edge", "k_photo", "k_schur", "k_solve", "k_sinv_helper",
              "k_peer_push", "k_backsub", "k_project_error", "k_delay", "k_oc_step"):
        assert k in names, k


def test_group_kernels_two_waves_per_simd(kernels):
    for k, v in kernels.items():
        if "k_group" in k:
            assert int(v["vgpr_count"]) <= 256, (k, v)
