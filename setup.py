"""Build the penroz native extensions in-tree for gfx950 with hipcc (no hipify, no CUDA).

    python setup.py build_ext        # -> build_ext/penroz_kernels*.so, build_ext/penroz_comm*.so
    PENROZ_DEBUG=1 python setup.py build_ext   # -> build_ext/debug/ (-O1, device bounds
                                     #    checks; load with PENROZ_EXT_DIR=build_ext/debug)
    python setup.py isa KERNEL.hip   # -> build_ext/isa/KERNEL.s (gfx950 device assembly, for audits:
                                     #    VGPR/AGPR counts, spills, s_waitcnt placement)

Each ``csrc/kernels/*.hip`` is compiled with ``hipcc --offload-arch=gfx950`` in parallel and
linked together with the pybind11 bindings against PyTorch's own libraries (including the
HIP runtime PyTorch bundles, so exactly one ``libamdhip64`` is mapped in the process).
``csrc/comm/*.cpp`` (RCCL communicator) links PyTorch's bundled ``librccl``.
Objects are rebuilt only when a source or header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
DEBUG = os.environ.get("PENROZ_DEBUG", "0") == "1"
# PENROZ_BUILD_DIR overrides (A/B builds); debug builds default to build_ext/debug and are
# loaded with PENROZ_EXT_DIR=build_ext/debug
OUT = os.environ.get("PENROZ_BUILD_DIR") or os.path.join(ROOT, "build_ext", "debug" if DEBUG else "")
OUT = OUT.rstrip(os.sep)
OBJ = os.path.join(OUT, "obj")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    tdir = os.path.dirname(torch.__file__)
    return ce.include_paths(), os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _flags(name: str):
    incs, _, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    opt = ["-O1", "-DPENROZ_DEBUG=1"] if DEBUG else ["-O3"]
    f = opt + ["-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-D__HIP_PLATFORM_AMD__=1",
         "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-DTORCH_EXTENSION_NAME={name}",
         "-DTORCH_API_INCLUDE_EXTENSION_H", "-Wno-unused-result", "-Wno-unused-variable",
         "-Wno-deprecated-declarations", f"-I{py_inc}", f"-I{CSRC}", f"-I{os.path.join(CSRC, 'kernels')}"]
    f += [f"-I{p}" for p in incs]
    return f


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _newer(src: str, obj: str, deps: list[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src] + deps)


def _compile(src: str, obj: str, flags: list[str]):
    cmd = [HIPCC] + flags + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build_module(name: str, sources: list[str], extra_libs: list[str], jobs: int) -> str:
    os.makedirs(OBJ, exist_ok=True)
    flags = _flags(name)
    headers = [os.path.join(CSRC, "kernels", h) for h in os.listdir(os.path.join(CSRC, "kernels")) if h.endswith(".h")]
    todo = []
    objs = []
    for s in sources:
        obj = os.path.join(OBJ, f"{name}__{os.path.basename(s)}.o")
        objs.append(obj)
        if _newer(s, obj, headers):
            todo.append((s, obj))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for fut in cf.as_completed([ex.submit(_compile, s, o, flags) for s, o in todo]):
            print(f"[build] compiled {os.path.basename(fut.result())}", flush=True)
    _, tlib, _ = _torch_paths()
    target = os.path.join(OUT, name + _ext_suffix())
    if todo or not os.path.exists(target):
        tmp = target + ".tmp"  # link aside, then rename: a snapshot of the tree never sees half a .so
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + [
            f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            "-lamdhip64", f"-Wl,-rpath,{tlib}"] + extra_libs
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed for {name}\n{' '.join(link)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, target)
        print(f"[build] linked {target}", flush=True)
    return target


def build_all(jobs: int | None = None) -> list[str]:
    jobs = jobs or min(8, os.cpu_count() or 4)
    kdir = os.path.join(CSRC, "kernels")
    ksrc = sorted(os.path.join(kdir, f) for f in os.listdir(kdir) if f.endswith(".hip"))
    ksrc.append(os.path.join(CSRC, "bindings.cpp"))
    built = [build_module("penroz_kernels", ksrc, [], jobs)]
    cdir = os.path.join(CSRC, "comm")
    csrc = sorted(os.path.join(cdir, f) for f in os.listdir(cdir) if f.endswith(".cpp")) if os.path.isdir(cdir) else []
    if csrc:
        _, tlib, _ = _torch_paths()
        built.append(build_module("penroz_comm", csrc, [f"{tlib}/librccl.so"], jobs))
    return built


def dump_isa(src_name: str) -> str:
    """Device assembly of one kernel source (``--cuda-device-only -S``)."""
    src = os.path.join(CSRC, "kernels", src_name)
    out_dir = os.path.join(OUT, "isa")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, os.path.splitext(src_name)[0] + ".s")
    cmd = [HIPCC] + _flags("penroz_kernels") + ["--cuda-device-only", "-S", src, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"isa dump failed: {src}\n{r.stderr}")
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "isa":
        for name in sys.argv[2:]:
            print(dump_isa(name))
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] not in ("build_ext", "build"):
        print(__doc__)
        sys.exit(2)
    for p in build_all():
        print(p)
