#!/usr/bin/env python3
"""Interleaved A/B timing of library variants: tools/ab.py rounds lib1.so lib2.so ... [-- K N B G]"""
import os, subprocess, sys
args = sys.argv[1:]
shape = []
if "--" in args:
    i = args.index("--"); shape = args[i + 1:]; args = args[:i]
rounds = int(args[0]); libs = args[1:]
here = os.path.dirname(os.path.abspath(__file__))
for r in range(rounds):
    for spec in libs:
        lib, _, kv = spec.partition(":")  # lib.so[:KEY=VAL,KEY=VAL]
        env = dict(os.environ, KFEC_LIB=os.path.abspath(lib))
        for item in filter(None, kv.split(",")):
            k, v = item.split("=", 1)
            env[k] = v
        p = subprocess.run([sys.executable, os.path.join(here, "ab_one.py")] + shape, env=env,
                           capture_output=True, text=True, timeout=600)
        print(spec.split("/")[-1], p.stdout.strip() or p.stderr[-2000:], flush=True)
        if p.returncode != 0:
            sys.exit(p.returncode)
