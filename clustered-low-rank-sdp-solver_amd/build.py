"""Build libclrsdp.so in-tree with hipcc for gfx950 (no CMake; one translation unit)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "clrsdp.hip")
OUT = os.path.join(HERE, "libclrsdp.so")
DEPS = [SRC, os.path.join(HERE, "csrc", "kernels.h"), os.path.join(HERE, "csrc", "mwfloat.h"),
        os.path.join(HERE, "csrc", "kernels_dense.h"),
        os.path.join(HERE, "..", "include", "clrsdp.h")]

HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               # keep MFMA accumulators in the unified VGPR file (otherwise hipcc shuttles them
               # through AGPRs every k-step: 46.7 vs 72.4 TF/s fp64, profiles/r01_f64_mfma_probe.log)
               "-mllvm", "-amdgpu-mfma-vgpr-form", "-ldl"]


def source_hash() -> str:
    """sha256 over the library's sources (csrc + the C ABI header): names the build a profile or
    counter pass was taken on, so results of another build are recognised as stale."""
    import hashlib
    h = hashlib.sha256()
    for d in DEPS:
        with open(d, "rb") as f:
            h.update(os.path.basename(d).encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


# the compiler's per-kernel resource remarks of the last build (VGPRs, scratch, occupancy), kept
# beside the library for tests/test_build_resources.py (a kernel that starts spilling to scratch
# is a silent slowdown: round 6 found schur_fused_f64 at 92 B/lane after an epilogue change)
RESOURCES = os.path.join(HERE, "libclrsdp.resources.txt")


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and os.path.exists(OUT):
        t = os.path.getmtime(OUT)
        if all(os.path.getmtime(d) <= t for d in DEPS if os.path.exists(d)):
            return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc] + HIPCC_FLAGS + ["-Rpass-analysis=kernel-resource-usage", "-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, stderr=subprocess.PIPE, text=True)
    with open(RESOURCES + ".tmp", "w") as f:
        f.write(r.stderr)
    if r.returncode != 0:
        print("\n".join(ln for ln in r.stderr.splitlines() if "remark:" not in ln), file=sys.stderr)
        raise subprocess.CalledProcessError(r.returncode, cmd)
    os.replace(RESOURCES + ".tmp", RESOURCES)
    os.replace(OUT + ".tmp", OUT)
    return OUT


def kernel_resources(path: str = RESOURCES) -> dict:
    """{mangled kernel name: {"VGPRs": .., "ScratchSize": .., ...}} from the build's remarks."""
    out, cur = {}, None
    with open(path) as f:
        for ln in f:
            if "remark:" not in ln:
                continue
            body = ln.split("remark:", 1)[1].split("[-Rpass")[0].strip()
            if body.startswith("Function Name:"):
                cur = body.split(":", 1)[1].strip()
                out[cur] = {}
            elif cur is not None and ":" in body:
                k, v = body.split(":", 1)
                k = k.split("[")[0].strip()
                try:
                    out[cur][k] = int(v.strip())
                except ValueError:
                    pass
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
