#!/bin/bash
# One SQ counter pass over bench_seal.py for the shipped build and each kcptube_amd/variants/libkfec_seal_*.so
set -o pipefail
out=gpurun_out/seal_pmc; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in base $(cd kcptube_amd/variants && ls libkfec_seal_*.so | sed 's/libkfec_//; s/\.so//'); do
  lib=""; [ "$v" != base ] && lib=kcptube_amd/variants/libkfec_$v.so
  KFEC_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/$v -o p -- python3 tools/bench_seal.py --steps 1 --packets 1048576 > $out/$v.log 2>&1 || { tail $out/$v.log; exit 1; }
done
echo pmc-done
