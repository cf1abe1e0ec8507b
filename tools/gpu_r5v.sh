#!/bin/bash
# Round 5: VALU issue cost of the SDWA byte moves (isabench), then the OCB kernel with SDWA table addresses
# (shipped) against v_perm_b32 addresses (aead_ocbperm): AEAD GPU tests and an interleaved A/B.
set -o pipefail
out=gpurun_out/r5v; mkdir -p $out
timeout -k 10 120 ./tools/isabench > $out/isabench.txt 2>&1 || { cat $out/isabench.txt; exit 1; }
cat $out/isabench.txt
timeout -k 10 900 bash tools/gpu_aead_ab.sh > $out/ab.txt 2>&1 || { tail -30 $out/ab.txt; exit 1; }
cat $out/ab.txt
