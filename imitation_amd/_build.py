"""In-tree native build for ``imitation_amd._C``.

Layout (all MI355X / gfx950 only):

* ``csrc/kernels/*.hip``  — HIP/CDNA4 kernels + their host launchers
  (``hipcc --offload-arch=gfx950``; no torch headers, so they compile in seconds);
* ``csrc/runtime/*.cpp``  — native host runtime (batched envs, ...), plain
  ``g++ -fopenmp``; the env dynamics headers are ``__host__ __device__`` and
  shared verbatim with the device rollout kernel;
* ``csrc/bind/*.cpp``  — the only TUs that see torch/pybind11 headers
  (``g++``), turning tensors into raw pointers + the current HIP stream.

Objects go to ``build/native``; the extension lands next to this file so it
ships with the repo snapshot to the GPU box. Rebuilds are incremental on
source / header mtimes.
"""

from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import json
import os
import shutil
import subprocess
import sys
import sysconfig
from typing import List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
PKG = os.path.join(ROOT, "imitation_amd")
EXT_NAME = "_C"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = "gfx950"


def ext_path() -> str:
    return os.path.join(PKG, EXT_NAME + sysconfig.get_config_var("EXT_SUFFIX"))


def _torch_paths():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return tdir, inc, os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _sources():
    kernels = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    runtime = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    bindings = sorted(glob.glob(os.path.join(CSRC, "bind", "*.cpp")))
    return kernels, runtime, bindings


def _headers() -> List[str]:
    return sorted(
        glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
        + glob.glob(os.path.join(CSRC, "**", "*.hpp"), recursive=True)
        + glob.glob(os.path.join(CSRC, "**", "*.cuh"), recursive=True)
    )


def _flags():
    _, tinc, tlib, abi = _torch_paths()
    common_inc = [f"-I{os.path.join(CSRC, 'include')}", f"-I{os.path.join(CSRC, 'kernels')}", f"-I{os.path.join(CSRC, 'runtime')}"]
    hip = [
        os.path.join(ROCM, "bin", "hipcc"),
        f"--offload-arch={ARCH}",
        "-O3",
        "-fPIC",
        "-std=c++17",
        "-munsafe-fp-atomics",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-Wno-unused-result",
    ] + common_inc
    host_cxx = [
        "g++",
        "-O3",
        "-fPIC",
        "-std=c++17",
        "-fopenmp",
        "-D__HIP_PLATFORM_AMD__=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        f"-I{os.path.join(ROCM, 'include')}",
    ] + common_inc
    py_inc = sysconfig.get_paths()["include"]
    gxx = [
        "g++",
        "-O2",
        "-fPIC",
        "-std=c++17",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        f"-DTORCH_EXTENSION_NAME={EXT_NAME}",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        f"-I{py_inc}",
        f"-I{os.path.join(ROCM, 'include')}",
    ] + [f"-I{p}" for p in tinc] + common_inc
    link = [
        "g++",
        "-shared",
        "-fopenmp",
        f"-L{tlib}",
        f"-Wl,-rpath,{tlib}",
        "-lc10",
        "-ltorch",
        "-ltorch_cpu",
        "-ltorch_python",
        "-lc10_hip",
        "-ltorch_hip",
        "-lamdhip64",
        f"-L{os.path.join(ROCM, 'lib')}",
    ]
    return hip, host_cxx, gxx, link


def _obj_name(src: str) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(BUILD, rel + ".o")


def _needs_build(src: str, obj: str, hdr_mtime: float, flags_sig: str) -> bool:
    if not os.path.exists(obj):
        return True
    sig = obj + ".sig"
    if not os.path.exists(sig) or open(sig).read() != flags_sig:
        return True
    m = os.path.getmtime(obj)
    return os.path.getmtime(src) > m or hdr_mtime > m


def _compile(cmd: List[str], obj: str, sig: str, verbose: bool) -> Optional[str]:
    if verbose:
        print(" ".join(cmd), flush=True)
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        return f"FAILED: {' '.join(cmd)}\n{proc.stdout}\n{proc.stderr}"
    with open(obj + ".sig", "w") as f:
        f.write(sig)
    return None


def build(force: bool = False, verbose: bool = False, jobs: Optional[int] = None) -> str:
    """Compile every HIP kernel + runtime TU for gfx950 and link ``imitation_amd._C``."""
    os.makedirs(BUILD, exist_ok=True)
    hip, host_cxx, gxx, link = _flags()
    kernels, runtime, bindings = _sources()
    hdrs = _headers()
    hdr_mtime = max([os.path.getmtime(h) for h in hdrs] + [0.0])
    jobs_list = []
    for src in kernels:
        obj = _obj_name(src)
        cmd = hip + ["-c", src, "-o", obj]
        jobs_list.append((src, obj, cmd))
    for src in runtime:
        obj = _obj_name(src)
        cmd = host_cxx + ["-c", src, "-o", obj]
        jobs_list.append((src, obj, cmd))
    for src in bindings:
        obj = _obj_name(src)
        cmd = gxx + ["-c", src, "-o", obj]
        jobs_list.append((src, obj, cmd))
    todo = []
    for src, obj, cmd in jobs_list:
        sig = hashlib.sha1(json.dumps(cmd).encode()).hexdigest()
        if force or _needs_build(src, obj, hdr_mtime, sig):
            todo.append((cmd, obj, sig))
    n_jobs = jobs or min(len(todo) or 1, max(1, min(16, (os.cpu_count() or 4))))
    errors = []
    if todo:
        with cf.ThreadPoolExecutor(n_jobs) as ex:
            for err in ex.map(lambda t: _compile(t[0], t[1], t[2], verbose), todo):
                if err:
                    errors.append(err)
    if errors:
        raise RuntimeError("native build failed:\n" + "\n".join(errors))
    out = ext_path()
    objs = [o for _, o, _ in jobs_list]
    newest = max(os.path.getmtime(o) for o in objs)
    if force or todo or not os.path.exists(out) or os.path.getmtime(out) < newest:
        tmp = out + ".tmp"
        cmd = link[:2] + objs + ["-o", tmp] + link[2:]
        if verbose:
            print(" ".join(cmd), flush=True)
        proc = subprocess.run(cmd, capture_output=True, text=True)
        if proc.returncode != 0:
            raise RuntimeError(f"link failed:\n{proc.stdout}\n{proc.stderr}")
        os.replace(tmp, out)
    return out


def is_stale() -> bool:
    out = ext_path()
    if not os.path.exists(out):
        return True
    m = os.path.getmtime(out)
    kernels, runtime, bindings = _sources()
    return any(os.path.getmtime(p) > m for p in kernels + runtime + bindings + _headers())


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose="-v" in sys.argv))
