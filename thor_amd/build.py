"""Build libthor_amd.so in-tree with hipcc for gfx950 (no JIT cache: the .so
travels to the GPU box with the repository snapshot)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libthor_amd.so")
# every translation unit and header under csrc/ (libthor_amd.hip #includes the .hip files)
SOURCES = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".h")))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-Wall", "-Wno-unused-result", "-Wno-bitwise-instead-of-logical"]
# Integer dot products as the three-operand VOP3P forms (v_dot4_i32_i8, v_dot2_i32_i16):
# with the accumulate-in-place VOP2 forms (v_dot4c / v_dot2c) available hipcc seeds every
# chain with a v_mov (k_recon: ~3 700 of them).  The host pass ignores these (it warns).
FLAGS += ["-Xclang", "-target-feature", "-Xclang", "-dot6-insts", "-Xclang", "-target-feature", "-Xclang", "-dot4-insts"]
# k_recon: 5 waves per SIMD (96 VGPRs; a few spills on the per-cell path only)
FLAGS += ["-DRECON_WPE=5"]
# No interprocedural register allocation: with it (the AMDGPU default) a caller of
# the encoder's non-inlined RD functions allocates against each callee's actual
# clobber set, and a register-hungry callee (the candidate-parallel motion search)
# turned the callers' values into spill / reload traffic around every call (the
# 4K I frame, which never runs that callee, +8 %).  Without it every function
# keeps the calling convention's contract: 240 x 4K I frame 1 270 -> 1 173 ms.
FLAGS += ["-mllvm", "-enable-ipra=false"]


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(HERE, "..", "include", "thor_amd.h"),
                                                      os.path.join(HERE, "..", "include", "thor_kernels.h")]
    return any(os.path.exists(p) and os.path.getmtime(p) > t for p in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if force or _stale():
        cmd = [HIPCC] + FLAGS + ["-o", LIB, os.path.join(CSRC, "libthor_amd.hip")]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True, cwd=CSRC)
    return LIB


if __name__ == "__main__":
    build(force=True, verbose=True)
