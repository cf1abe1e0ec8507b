#!/bin/bash
# A/B of seal/open builds: tools/ab_seal.sh lib1.so lib2.so ...
for v in "$@"; do
  echo $v; KFEC_LIB=$PWD/$v timeout -k 10 120 python tools/bench_seal.py --steps 5 || exit 1
done
