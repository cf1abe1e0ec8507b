#!/usr/bin/env python3
"""Build a timing / ablation variant of libkfec.so on the CPU (before a tools/gpu_ab.sh call):

    python tools/build_variant.py <name> KEY=VAL [KEY=VAL ...] [--flags <source>:<flag>[,<flag>...]]

writes kcptube_amd/variants/libkfec_<name>.so, the shipped sources with -DKEY=VAL (the compile-time knobs at the
top of kcptube_amd/csrc/*.hip, e.g. KFEC_XCD_ORDER=4, KFEC_SYN_XORONLY=1) and optional extra per-source compiler
flags (e.g. --flags kfec_kernels.hip:-mllvm,-amdgpu-sched-strategy=iterative-minreg).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kcptube_amd.build import build_variant  # noqa: E402


def main(argv):
    if not argv or "=" in argv[0]:
        raise SystemExit(__doc__)
    name, defines, flags = argv[0], {}, {}
    it = iter(argv[1:])
    for a in it:
        if a == "--flags":
            src, _, fl = next(it).partition(":")
            flags.setdefault(src, []).extend(f for f in fl.split(",") if f)
        else:
            k, _, v = a.partition("=")
            defines[k] = int(v, 0)
    print(build_variant(name, defines, flags))


if __name__ == "__main__":
    main(sys.argv[1:])
