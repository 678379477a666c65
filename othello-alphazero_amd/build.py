"""Build the MI355X-native othello_mcts extension in-tree.

  liboamd.so               HIP kernels (tree.hip, resnet.hip) + the C ABI (capi.hip),
                           hipcc --offload-arch=gfx950
  _othello_mcts_impl*.so   pybind11 host layer (pybind_module.cpp) over the C ABI

Both land in othello-alphazero_amd/othello_mcts/ (git-ignored, shipped to the
GPU box with the snapshot). Usage: python othello-alphazero_amd/build.py [-j N]
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
PKG = HERE / "othello_mcts"
INCLUDE = HERE.parent / "include"
BUILD = HERE / "build"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("OAMD_ARCH", "gfx950")

COMMON = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", str(CSRC), "-I", str(INCLUDE),
          "-Wall", "-Wno-unused-function", "-fno-gpu-rdc", *os.environ.get("OAMD_EXTRA_FLAGS", "").split()]
# tree.hip / rng.h / capi.hip tables must reproduce the reference's float
# arithmetic bit for bit: no FMA contraction, IEEE division and sqrt.
EXACT = ["-ffp-contract=off", "-fno-fast-math"]
# tree.hip's kernels read statistics, links and game state that the same wave
# has just written with vector stores (ordered by a wavefront fence, tree.hip
# wave_order): no global load may go through the scalar cache, which does not
# see those stores (tests/test_cpu_host.py checks the ISA)
NO_SCALAR_LOADS = ["-mllvm", "-amdgpu-scalarize-global-loads=false"]
UNITS = {
    "tree.hip": EXACT + NO_SCALAR_LOADS,
    "capi.hip": EXACT,
    # accumulators and fragments in arch VGPRs: the default heuristic parks the
    # 128 accumulators of a 1-wave/SIMD tile in AGPRs and shuffles them per MFMA;
    # the max-ILP machine scheduler: k_resnet_w8 0.895-0.900 vs 0.907-0.913 ms per
    # 4096 rows (3 same-box pairs, outputs bit-identical; tools/ab_run1.sh)
    "resnet.hip": os.environ.get("OAMD_RESNET_FLAGS",
                                 "-mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-sched-strategy=max-ilp").split()
    + ["-Rpass-analysis=kernel-resource-usage"],
}


# k_resnet_w8 (8 waves, 2 per SIMD) must allocate <= 208 VGPRs per wave so one
# k_select wave (93 VGPRs) still fits beside it on each SIMD (resnet.hip)
W8_VGPR_LIMIT = 208


def run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise SystemExit(f"build failed: {cmd[-1]}")
    if "kernel-resource-usage" in " ".join(cmd):
        check_w8_vgprs(r.stderr)
    elif r.stderr.strip():
        sys.stderr.write(r.stderr)


def check_w8_vgprs(remarks: str) -> None:
    """Parse -Rpass-analysis=kernel-resource-usage remarks; fail if a k_resnet_w8
    instantiation's VGPR allocation (granule 8) exceeds W8_VGPR_LIMIT."""
    name = None
    seen = 0
    for ln in remarks.splitlines():
        if "Function Name:" in ln:
            name = ln.split("Function Name:")[1].split()[0]
        elif name and "k_resnet_w8" in name and " VGPRs:" in ln:
            v = int(ln.split("VGPRs:")[1].split()[0])
            seen += 1
            if (v + 7) // 8 * 8 > W8_VGPR_LIMIT and os.environ.get("OAMD_W8_VGPR_CHECK", "1") != "0":
                raise SystemExit(f"build failed: {name} uses {v} VGPRs (> {W8_VGPR_LIMIT}): "
                                 "k_select could no longer co-reside with the ResNet kernel")
    if not seen:  # A/B builds with other geometries (e.g. -DOAMD_WC=128) have no w8 kernel
        sys.stderr.write("note: no k_resnet_w8 kernel in this build\n")


def newer(out: Path, deps: list[Path]) -> bool:
    return out.exists() and all(out.stat().st_mtime >= d.stat().st_mtime for d in deps)


def source_hash_defines() -> list[str]:
    """-D flags carrying the source hashes (othello_mcts/provenance.py) into
    capi.hip, so the library reports what it was built from."""
    sys.path.insert(0, str(PKG))
    try:
        import provenance
    finally:
        sys.path.pop(0)
    return [f'-DOAMD_SOURCE_HASH_{k.upper()}="{provenance.source_hash(k)}"' for k in provenance.FAMILIES]


def build(jobs: int = 4, force: bool = False) -> None:
    BUILD.mkdir(exist_ok=True)
    headers = list(CSRC.glob("*.h")) + [INCLUDE / "othello_mcts_amd.h", INCLUDE / "othello_mcts_amd_experimental.h"]
    hashes = source_hash_defines()
    objs = []
    todo = []
    all_srcs = [CSRC / u for u in UNITS] + headers
    for unit, extra in UNITS.items():
        src = CSRC / unit
        obj = BUILD / (unit + ".o")
        objs.append(obj)
        # capi.hip carries the hashes of every source: rebuilt when any changes
        deps = all_srcs if unit == "capi.hip" else [src, *headers]
        if force or not newer(obj, [*deps, Path(__file__)]):
            todo.append([HIPCC, *COMMON, *extra, *(hashes if unit == "capi.hip" else []), "-c", str(src),
                         "-o", str(obj)])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(run, todo))
    lib = PKG / "liboamd.so"
    if force or todo or not lib.exists():
        run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib), *map(str, objs)])

    # pybind11 host layer: plain C++ against the C ABI, no torch headers
    import pybind11

    ext = sysconfig.get_config_var("EXT_SUFFIX")
    mod = PKG / f"_othello_mcts_impl{ext}"
    src = CSRC / "pybind_module.cpp"
    if force or not newer(mod, [src, *headers, lib, Path(__file__)]):
        run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-fvisibility=hidden",
             "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"], "-I", str(INCLUDE),
             str(src), "-o", str(mod), "-L", str(PKG), "-loamd", "-Wl,-rpath,$ORIGIN"])


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=4)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    build(a.jobs, a.force)
    print("built", *sorted(p.name for p in PKG.glob("*.so")))
