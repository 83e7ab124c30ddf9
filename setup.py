"""Build the p2pfl_amd native extension in-tree for MI355X (gfx950).

    python setup.py build_ext --inplace

Kernels (``csrc/*.hip``) are compiled directly by ``hipcc --offload-arch=gfx950``
into position-independent objects -- no hipify pass, no CUDA headers -- and
linked with the host-only PyTorch bindings (``csrc/*.cpp``) into
``p2pfl_amd/_C*.so`` next to the sources (the .so travels with the repository
snapshot to GPU boxes; nothing is installed into site-packages).
"""

import glob
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

from setuptools import find_packages, setup
import torch
from torch.utils.cpp_extension import BuildExtension, CppExtension

HERE = os.path.dirname(os.path.abspath(__file__))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
# RCCL: link the copy PyTorch ships (same soname, already loaded by torch), so
# the data plane and torch.distributed share one library instance.
TORCH_LIB = os.path.join(os.path.dirname(torch.__file__), "lib")
OBJ_DIR = os.path.join(HERE, "build", "hipobj")
HIP_FLAGS = [
    "-O3",
    f"--offload-arch={ARCH}",
    "-std=c++17",
    "-fPIC",
    "-ffp-contract=fast",
    "-munsafe-fp-atomics",
    "-fno-gpu-rdc",
    "-I" + os.path.join(HERE, "csrc"),
]


def _compile_one(src: str) -> str:
    os.makedirs(OBJ_DIR, exist_ok=True)
    deps = [src] + sorted(glob.glob(os.path.join(HERE, "csrc", "*.h")))
    h = hashlib.sha1()
    for d in deps:
        with open(d, "rb") as f:
            h.update(f.read())
    h.update(" ".join(HIP_FLAGS).encode())
    obj = os.path.join(OBJ_DIR, os.path.basename(src) + "." + h.hexdigest()[:12] + ".o")
    if not os.path.exists(obj):
        cmd = [os.path.join(ROCM, "bin", "hipcc"), *HIP_FLAGS, "-c", src, "-o", obj]
        print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
    return obj


def hip_objects():
    srcs = sorted(glob.glob(os.path.join(HERE, "csrc", "*.hip")))
    jobs = int(os.environ.get("MAX_JOBS", "8"))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        return list(ex.map(_compile_one, srcs))


def host_libs():
    """Plain C ABI host libraries (no torch / HIP), loaded with ctypes."""
    src = os.path.join(HERE, "csrc", "host", "wire_frame.cpp")
    out = os.path.join(HERE, "p2pfl_amd", "_p2fa.so")
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(src), os.path.getmtime(src[:-4] + ".h")):
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wextra", src, "-o", out]
        print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)


class HipBuild(BuildExtension):
    def build_extensions(self):
        host_libs()
        objs = hip_objects()
        for ext in self.extensions:
            ext.extra_objects = list(ext.extra_objects or []) + objs
        super().build_extensions()


setup(
    name="p2pfl_amd",
    version="0.1.0",
    packages=find_packages(include=["p2pfl_amd", "p2pfl_amd.*"]),
    package_data={"p2pfl_amd.tuning": ["*.csv"], "p2pfl_amd": ["_p2fa.so"]},
    ext_modules=[
        CppExtension(
            "p2pfl_amd._C",
            sorted(glob.glob(os.path.join("csrc", "*.cpp"))),
            include_dirs=[os.path.join(HERE, "csrc"), os.path.join(ROCM, "include")],
            define_macros=[("__HIP_PLATFORM_AMD__", "1"), ("USE_ROCM", "1")],
            library_dirs=[TORCH_LIB, os.path.join(ROCM, "lib")],
            libraries=["amdhip64", "c10_hip", "torch_hip", "rccl"],
            extra_link_args=["-Wl,-rpath," + TORCH_LIB],
            extra_compile_args=["-O3", "-std=c++17"],
        )
    ],
    cmdclass={"build_ext": HipBuild.with_options(use_ninja=True)},
    entry_points={"console_scripts": ["p2pfl-amd=p2pfl_amd.cli:app"]},
)
