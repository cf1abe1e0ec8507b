"""Build libkfec.so (gfx950 HIP kernels + C ABI) in-tree with hipcc.

    python -m kcptube_amd.build          # or __graft_entry__.build()

The library lands at kcptube_amd/libkfec.so (git-ignored, but it travels to the GPU box with the
repo snapshot).  A C++ example/test of the fecpp::fec_code drop-in header is built alongside.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libkfec.so")
COMPAT_TEST = os.path.join(PKG, "compat_test")

SOURCES = ["kfec_kernels.hip", "kfec_frame.hip", "kfec_seal.hip", "kfec_aead.hip", "kfec_gcm.hip", "kfec_ocb.hip", "kfec_worker.hip", "kfec_api.cpp", "kfec_pipeline.cpp"]
HEADERS = ["kfec_gf.hpp", "kfec_internal.hpp", "kfec_count.hpp", "kfec_xcd.hpp", "kfec_aes.hpp", "kfec_pkt.hpp"]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: libkfec.so cannot be built")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


# per-source compiler flags of the shipped library.  kfec_ocb.hip: LLVM's iterative ILP scheduler keeps more of a
# round's table reads in flight (aes_ocb seal 8.31-8.33 -> 8.16 ms, profiles/r05_ocb_sched_ab.txt); applied to
# that file only (the same flag crashes the compiler on kfec_kernels.hip)
FILE_FLAGS: dict[str, list[str]] = {"kfec_ocb.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]}


def _compile_link(out: str, common: list[str], file_flags: dict[str, list[str]], verbose: bool = False,
                  link_extra: list[str] | None = None) -> None:
    """Each source to an object (in parallel, so a source can carry flags of its own), then one link."""
    import concurrent.futures
    import tempfile
    base = [_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result"] + common
    with tempfile.TemporaryDirectory(prefix="kfec_build_") as tmp:
        def one(src: str) -> str:
            obj = os.path.join(tmp, src + ".o")
            cmd = base + file_flags.get(src, []) + ["-c", "-o", obj, os.path.join(CSRC, src)]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.check_call(cmd, cwd=CSRC)
            return obj
        jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", "8"))))
        with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
            objs = list(ex.map(one, SOURCES))
        subprocess.check_call([_hipcc(), "--offload-arch=gfx950", "-fPIC", "-shared", "-o", out] + objs + (link_extra or []),
                              cwd=CSRC)


def build_lib(force: bool = False, verbose: bool = False) -> str:
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [os.path.join(ROOT, "include", h) for h in ("kfec.h", "kfec_frame.h", "kfec_pipeline.h", "kfec_aead.h")]
    if force or _stale(LIB, deps):
        _compile_link(LIB + ".tmp", [], FILE_FLAGS, verbose)
        os.replace(LIB + ".tmp", LIB)
    return LIB


def build_variant(name: str, defines: dict[str, int], flags: dict[str, list[str]] | None = None) -> str:
    """Timing/ablation variant of the library (tools/ab.py): kcptube_amd/variants/libkfec_<name>.so.
    `flags` maps a source file to extra compiler flags (on top of the shipped library's)."""
    out_dir = os.path.join(PKG, "variants")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, f"libkfec_{name}.so")
    ff = {k: list(v) for k, v in FILE_FLAGS.items()}
    for k, v in (flags or {}).items():
        ff[k] = ff.get(k, []) + list(v)
    _compile_link(out, [f"-D{k}={v}" for k, v in defines.items()], ff)
    return out


def build_tools(force: bool = False) -> list[str]:
    """The C++ programs over the public headers: tools/pipeline_bench (kfec_pipeline.h from C++, one
    sender + receiver per host thread, bit-exact recovery check; also run by tests/test_gpu_pipeline.py) and
    tools/latency_bench (the per-call latency path) and tools/worker_check (single calls through the resident
    worker, in a given order)."""
    inc = os.path.join(ROOT, "include")
    out = []
    for name, extra in (("pipeline_bench", ["-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include", "-L", "/opt/rocm/lib",
                                            "-lamdhip64", "-pthread"]),
                        ("latency_bench", ["-ldl"]), ("worker_check", []),
                        ("side_effects", ["-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include", "-L", "/opt/rocm/lib",
                                          "-lamdhip64", "-pthread"])):
        src = os.path.join(ROOT, "tools", name + ".cpp")
        exe = os.path.join(ROOT, "tools", name)
        deps = [src, LIB] + [os.path.join(inc, h) for h in ("kfec.h", "kfec_frame.h", "kfec_pipeline.h", "kfec_aead.h")]
        if force or _stale(exe, deps):
            cmd = ["g++", "-std=c++17", "-O2", "-I", inc, src, "-o", exe, "-L", PKG, "-lkfec",
                   "-Wl,-rpath,$ORIGIN/../kcptube_amd"] + extra
            subprocess.check_call(cmd)
        out.append(exe)
    # tools/libkfec_calib.so: the on-box read and GF-MAC VALU ceilings bench.py reports against
    src = os.path.join(ROOT, "tools", "calib.hip")
    so = os.path.join(ROOT, "tools", "libkfec_calib.so")
    if force or _stale(so, [src, os.path.join(CSRC, "kfec_gf.hpp")]):
        subprocess.check_call([_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                               "-Wno-unused-result", src, "-o", so + ".tmp"])
        os.replace(so + ".tmp", so)
    out.append(so)
    # tools/libkfec_arithfree.so: the shipped sources with every GF multiply-accumulate of the MAC and syndrome
    # kernels replaced by a plain XOR of the shard granules (no table reads) -- the same grids (XCD spans), loads and
    # stores, wrong results.  bench.py times its encode / decode in the same run as the ceiling of the product's own
    # access pattern (measurement only; -Bsymbolic: its C ABI binds to itself when both libraries are loaded)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    af = os.path.join(ROOT, "tools", "libkfec_arithfree.so")
    if force or _stale(af, deps):
        # (-Dkfec=kfec_af: its kernels are kfec_af::..., so a rocprofv3 trace of bench.py keeps them apart from the
        # product's kernels of the same name)
        _compile_link(af + ".tmp", ["-DKFEC_MAC_XORONLY=1", "-DKFEC_SYN_XORONLY=2", "-Dkfec=kfec_af"], FILE_FLAGS,
                      link_extra=["-Wl,-Bsymbolic"])
        os.replace(af + ".tmp", af)
    out.append(af)
    # tools/ceiling: the XOR-only HBM calibration kernels, also the FETCH_SIZE / WRITE_SIZE
    # calibration target of tools/gpu_profile_all.sh, so it must exist in the tree that travels to the box
    src = os.path.join(ROOT, "tools", "ceiling.hip")
    exe = os.path.join(ROOT, "tools", "ceiling")
    if os.path.exists(src) and (force or _stale(exe, [src])):
        subprocess.check_call([_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-unused-result",
                               "-Wno-unused-value", src, "-o", exe])
    out.append(exe)
    # tools/cpu_aead: the OpenSSL CPU leg of tools/bench_aead.py (skipped where the OpenSSL headers are absent)
    src = os.path.join(ROOT, "tools", "cpu_aead.c")
    exe = os.path.join(ROOT, "tools", "cpu_aead")
    if os.path.exists(src) and os.path.exists("/usr/include/openssl/evp.h") and (force or _stale(exe, [src])):
        subprocess.check_call(["gcc", "-O2", "-pthread", "-o", exe, src, "-lcrypto"])
        out.append(exe)
    return out


def build_compat_test(force: bool = False) -> str:
    """C++ program exercising include/fecpp_compat.hpp against libkfec.so (run by the GPU tests)."""
    src = os.path.join(ROOT, "tests", "cpp", "compat_test.cpp")
    deps = [src, os.path.join(ROOT, "include", "fecpp_compat.hpp"), os.path.join(ROOT, "include", "kfec.h"), LIB]
    if force or _stale(COMPAT_TEST, deps):
        cmd = ["g++", "-std=c++20", "-O2", "-I", os.path.join(ROOT, "include"), src, "-o", COMPAT_TEST,
               "-L", PKG, "-lkfec", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath," + PKG]
        subprocess.check_call(cmd)
    return COMPAT_TEST


def main() -> None:
    force = "--force" in sys.argv
    print(build_lib(force=force, verbose=True))
    if os.path.exists(os.path.join(ROOT, "tests", "cpp", "compat_test.cpp")):
        print(build_compat_test(force=force))


if __name__ == "__main__":
    main()
