"""Build the native module akka_allreduce_1_amd/_C (C++17 runtime + HIP/CDNA4 kernels).

Pure C++ sources (protocol cores, actor runtime, TCP cluster transport, bindings) are
compiled with g++; `.hip` sources with hipcc for gfx950 only. Objects are cached under
build/native and rebuilt when the source or any header under csrc/ changes. The module
is linked in-tree so it travels to the GPU box with the repository snapshot.

usage: python tools/build_native.py [-j N] [--clean] [--debug] [--sanitize=thread|address]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "csrc"
PKG = ROOT / "akka_allreduce_1_amd"
BUILD = ROOT / "build" / "native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _includes() -> list[str]:
    import pybind11

    return [
        f"-I{pybind11.get_include()}",
        f"-I{sysconfig.get_paths()['include']}",
        f"-I{CSRC}",
        f"-I{ROCM / 'include'}",
    ]


def _sources() -> list[Path]:
    srcs = []
    for sub in ("core", "runtime", "cluster", "bindings", "hip"):
        d = CSRC / sub
        if d.is_dir():
            srcs += sorted(p for p in d.iterdir() if p.suffix in (".cc", ".hip"))
    return srcs


def _headers_mtime() -> float:
    return max((p.stat().st_mtime for p in CSRC.rglob("*.h")), default=0.0)


def output_path() -> Path:
    return PKG / ("_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def exe_path() -> Path:
    """The native master/worker executable (csrc/tools/mxar_main.cc)."""
    return PKG / "mxar"


def _compile(src: Path, obj: Path, debug: bool, sanitize: str | None) -> tuple[Path, str]:
    opt = ["-O0", "-g"] if debug else ["-O3", "-DNDEBUG"]
    common = ["-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function"] + opt + _includes()
    common += ["-D__HIP_PLATFORM_AMD__"]
    if src.suffix == ".hip":
        cmd = [str(ROCM / "bin" / "hipcc"), "-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]
        cmd += common + ["-c", str(src), "-o", str(obj)]
        if sanitize:
            # host code only: GPU sanitizers are not available on the pool
            cmd += [f"-Xarch_host", f"-fsanitize={sanitize}"]
    else:
        cmd = [os.environ.get("CXX", "g++")] + common + ["-c", str(src), "-o", str(obj)]
        if sanitize:
            cmd += [f"-fsanitize={sanitize}", "-fno-omit-frame-pointer"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj, r.stderr


def build(jobs: int | None = None, clean: bool = False, debug: bool = False, sanitize: str | None = None,
          verbose: bool = True) -> Path:
    if clean and BUILD.exists():
        shutil.rmtree(BUILD)
    tag = ("dbg" if debug else "rel") + (f"-{sanitize}" if sanitize else "")
    bdir = BUILD / tag
    bdir.mkdir(parents=True, exist_ok=True)
    hdr = _headers_mtime()
    jobs = jobs or min(16, os.cpu_count() or 4)
    todo, objs = [], []
    for src in _sources():
        obj = bdir / (src.parent.name + "_" + src.name + ".o")
        objs.append(obj)
        if not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hdr):
            todo.append((src, obj))
    if todo:
        if verbose:
            print(f"[build_native] compiling {len(todo)} file(s) with -j{jobs}", flush=True)
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_compile, s, o, debug, sanitize) for s, o in todo]
            for f in cf.as_completed(futs):
                obj, err = f.result()
                if verbose:
                    print(f"  [ok] {obj.name}", flush=True)
                if err.strip() and verbose:
                    print(err, file=sys.stderr)
    out = output_path()
    if todo or not out.exists() or out.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        cmd = [str(ROCM / "bin" / "hipcc"), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(out)]
        cmd += [str(o) for o in objs]
        cmd += [f"-L{ROCM / 'lib'}", "-lamdhip64", "-lhsa-runtime64", "-lrocprofiler-sdk-roctx", f"-Wl,-rpath,{ROCM / 'lib'}", "-lpthread"]
        if sanitize:
            cmd += [f"-fsanitize={sanitize}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[build_native] linked {out.relative_to(ROOT)}", flush=True)
    if not sanitize:
        _build_exe(bdir, debug, verbose)
        _build_gpu_exe(bdir, debug, verbose)
    return out


def _build_exe(bdir: Path, debug: bool, verbose: bool) -> None:
    """Link the Python-free `mxar` executable from the host runtime objects (core, runtime,
    cluster) + csrc/tools/mxar_main.cc."""
    main_src = CSRC / "tools" / "mxar_main.cc"
    main_obj = bdir / "tools_mxar_main.cc.o"
    if not main_obj.exists() or main_obj.stat().st_mtime < max(main_src.stat().st_mtime, _headers_mtime()):
        _compile(main_src, main_obj, debug, None)
    objs = [bdir / (p.parent.name + "_" + p.name + ".o") for sub in ("core", "runtime", "cluster")
            for p in sorted((CSRC / sub).glob("*.cc"))] + [main_obj]
    exe = exe_path()
    if exe.exists() and exe.stat().st_mtime >= max(o.stat().st_mtime for o in objs):
        return
    cmd = [os.environ.get("CXX", "g++"), "-o", str(exe)] + [str(o) for o in objs]
    cmd += [f"-L{ROCM / 'lib'}", "-lrocprofiler-sdk-roctx", f"-Wl,-rpath,{ROCM / 'lib'}", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[build_native] linked {exe.relative_to(ROOT)}", flush=True)


def gpu_exe_path() -> Path:
    """The native worker with the round engine on a GPU (csrc/tools/mxar_gpu.cc)."""
    return PKG / "mxar-gpu"


def _build_gpu_exe(bdir: Path, debug: bool, verbose: bool) -> None:
    """Link `mxar-gpu`: the `mxar` objects + the HIP plane (every csrc/hip object except the
    Python bindings) + csrc/tools/mxar_gpu.cc, which resolves mxar_main's weak make_gpu_worker."""
    gpu_src = CSRC / "tools" / "mxar_gpu.cc"
    gpu_obj = bdir / "tools_mxar_gpu.cc.o"
    if not gpu_obj.exists() or gpu_obj.stat().st_mtime < max(gpu_src.stat().st_mtime, _headers_mtime()):
        _compile(gpu_src, gpu_obj, debug, None)
    hip = [bdir / ("hip_" + p.name + ".o") for p in sorted((CSRC / "hip").iterdir())
           if p.suffix in (".cc", ".hip") and not p.name.endswith("_bind.cc")]
    objs = [bdir / (p.parent.name + "_" + p.name + ".o") for sub in ("core", "runtime", "cluster")
            for p in sorted((CSRC / sub).glob("*.cc"))] + hip + [gpu_obj, bdir / "tools_mxar_main.cc.o"]
    exe = gpu_exe_path()
    if exe.exists() and exe.stat().st_mtime >= max(o.stat().st_mtime for o in objs):
        return
    cmd = [str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-o", str(exe)] + [str(o) for o in objs]
    cmd += [f"-L{ROCM / 'lib'}", "-lamdhip64", "-lhsa-runtime64", "-lrocprofiler-sdk-roctx", f"-Wl,-rpath,{ROCM / 'lib'}", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[build_native] linked {exe.relative_to(ROOT)}", flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--sanitize", choices=["thread", "address", "undefined"], default=None)
    a = ap.parse_args()
    build(a.j, a.clean, a.debug, a.sanitize)


if __name__ == "__main__":
    main()
