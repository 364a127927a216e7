"""Build driver for the native runtime (`nnstreamer_amd/_C*.so`).

Generates a ninja file that compiles every C++ source with hipcc (HIP
kernels for gfx950, the runtime as host C++), the PyTorch-ROCm filter
against libtorch, and links one in-tree Python extension.  No hipify, no
cpp_extension JIT: the .so is built in-tree so it travels with the repo.

    python nnstreamer_amd/_build.py [-j N] [--clean] [--verbose]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build")
ARCH = os.environ.get("NNSX_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("NNSX_CXX", "/opt/rocm/lib/llvm/bin/clang++")

# sources that include libtorch headers (slow to compile)
TORCH_SOURCES = {"filter/pytorch.cc", "filter/torch_trainer.cc", "filter/torch_lower.cc", "ops/torch_ops.cc"}
# pybind11 sources
PY_SOURCES = {"bindings/module.cc", "bindings/python_bridge.cc"}
# per-unit code generation: the x3 GEMMs keep MFMA results in VGPRs (kernels/gemm_f32.h)
UNIT_FLAGS = {"kernels/gemm_x3.hip": "-mllvm -amdgpu-mfma-vgpr-form", "kernels/irw_x3.hip": "-mllvm -amdgpu-mfma-vgpr-form",
              "kernels/irp_x3.hip": "-mllvm -amdgpu-mfma-vgpr-form"}


def ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def output_path() -> str:
    return os.path.join(ROOT, "nnstreamer_amd", "_C" + ext_suffix())


def runtime_lib_path() -> str:
    return os.path.join(ROOT, "nnstreamer_amd", "libnnsx.so")


# native command-line tools: csrc/tools/<name>.cc is part of libnnsx (entry
# point <name>_main); bin/<name with - for _> is csrc/tools/tool_main.cc built
# for that entry (it loads torch's HIP runtime, then libnnsx)
TOOLS = ("nnsx_launch", "nnsx_check")


def tool_path(name: str) -> str:
    return os.path.join(ROOT, "bin", name.replace("_", "-"))


def _sources():
    out = []
    for dp, _, files in os.walk(CSRC):
        for f in sorted(files):
            if f.endswith((".cc", ".hip")):
                rel = os.path.relpath(os.path.join(dp, f), CSRC)
                if rel == os.path.join("tools", "tool_main.cc"):
                    continue  # the executables' shim, linked separately
                out.append(rel)
    return sorted(out)


def _torch_paths():
    import torch  # noqa: F401  (only for include/library paths)
    from torch.utils import cpp_extension

    return cpp_extension.include_paths(), cpp_extension.library_paths()


def write_ninja(debug: bool = False) -> str:
    import pybind11

    os.makedirs(BUILD, exist_ok=True)
    tinc, tlib = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    opt = "-O0 -g" if debug else "-O3"
    common = f"{opt} -fPIC -std=c++17 -Wall -Wno-unused-function -Wno-unused-variable -Wno-sign-compare -I{CSRC} -I{ROOT}/include -D_GLIBCXX_USE_CXX11_ABI=1"
    hip_flags = f"-x hip --offload-arch={ARCH} -munsafe-fp-atomics -ffp-contract=fast"
    torch_flags = " ".join(f"-isystem {p}" for p in tinc) + " -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -Wno-deprecated-declarations -Wno-unknown-pragmas"
    py_flags = f"-isystem {pybind11.get_include()} -isystem {py_inc} -fvisibility=hidden"
    lib_dirs = " ".join(f"-L{p} -Wl,-rpath,{p}" for p in tlib)
    lines = [
        "ninja_required_version = 1.3",
        f"hipcc = {HIPCC}",
        f"cxx = {CXX}",
        f"common = {common}",
        "rule cxx",
        "  command = $cxx $common -D__HIP_PLATFORM_AMD__=1 -isystem /opt/rocm/include $extra -MMD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule hip",
        f"  command = $hipcc $common {hip_flags} $extra -MMD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIP $in",
        # the runtime (core, elements, kernels, filters, comm) as one shared library
        # the Python extension and the native tools link against
        "rule linklib",
        f"  command = $hipcc -shared -fPIC --offload-arch={ARCH} $in -o $out -Wl,-soname,libnnsx.so {lib_dirs} -ltorch -ltorch_cpu -ltorch_hip -lc10 -lc10_hip -lamdhip64 -L/opt/rocm/lib -lrccl -lrocprofiler-sdk-roctx -ldl -lpthread -Wl,--no-as-needed",
        "  description = LINK $out",
        "rule linkext",
        f"  command = $hipcc -shared -fPIC $in -o $out -L{ROOT}/nnstreamer_amd -lnnsx -Wl,-rpath,'$$ORIGIN' {lib_dirs} -ltorch -ltorch_cpu -lc10 -lamdhip64 -L/opt/rocm/lib -ldl -lpthread",
        "  description = LINK $out",
        "rule tool",
        f"  command = $cxx -O2 -std=c++17 -DNNSX_TOOL_ENTRY=$entry -DNNSX_TORCH_LIB='\"{tlib[0]}\"' $in -o $out -ldl",
        "  description = TOOL $out",
    ]
    lib_objs, py_objs = [], []
    for rel in _sources():
        obj = os.path.join(BUILD, rel.replace("/", "_") + ".o")
        extra = ""
        if rel in TORCH_SOURCES:
            extra = torch_flags
        if rel in PY_SOURCES:
            extra += " " + py_flags
        if rel in UNIT_FLAGS:
            extra += " " + UNIT_FLAGS[rel]
        rule = "hip" if rel.endswith(".hip") else "cxx"
        lines.append(f"build {obj}: {rule} {os.path.join(CSRC, rel)}")
        if extra:
            lines.append(f"  extra = {extra}")
        (py_objs if rel in PY_SOURCES else lib_objs).append(obj)
    lib = runtime_lib_path()
    lines.append(f"build {lib}: linklib {' '.join(lib_objs)}")
    lines.append(f"build {output_path()}: linkext {' '.join(py_objs)} | {lib}")
    outs = [lib, output_path()]
    for t in TOOLS:
        lines.append(f"build {tool_path(t)}: tool {os.path.join(CSRC, 'tools', 'tool_main.cc')}")
        lines.append(f"  entry = {t}_main")
        outs.append(tool_path(t))
    lines.append(f"default {' '.join(outs)}")
    path = os.path.join(BUILD, "build.ninja")
    content = "\n".join(lines) + "\n"
    old = open(path).read() if os.path.exists(path) else None
    if old != content:
        with open(path, "w") as f:
            f.write(content)
    return path


def _ninja() -> str:
    n = shutil.which("ninja")
    if n:
        return n
    import ninja  # pip wheel

    return os.path.join(ninja.BIN_DIR, "ninja")


def build(jobs: int | None = None, verbose: bool = False, debug: bool = False) -> str:
    write_ninja(debug=debug)
    if jobs is None:
        jobs = min(16, int(os.environ.get("MAX_JOBS", os.cpu_count() or 8)))
    cmd = [_ninja(), "-C", BUILD, "-j", str(jobs)]
    if verbose:
        cmd.append("-v")
    subprocess.check_call(cmd)
    return output_path()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--debug", action="store_true")
    a = ap.parse_args(argv)
    if a.clean and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    print(build(a.j, a.verbose, a.debug))


if __name__ == "__main__":
    sys.exit(main())
