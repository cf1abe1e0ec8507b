# round 4: aes_ocb with batched pad / tag enciphers -- AEAD parity, then A/B against the previous library
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_aead.py -x -q --timeout 300 --timeout-method thread > $O/aead.log 2>&1 || { tail -30 $O/aead.log; exit 1; }
tail -1 $O/aead.log
for lib in $V/libkfec_base.so kcptube_amd/libkfec.so $V/libkfec_base.so kcptube_amd/libkfec.so; do
  KFEC_LIB=$lib timeout -k 10 300 python tools/bench_aead.py --steps 5 >> $O/ab_aead.jsonl 2>> $O/ab_aead.err || { cat $O/ab_aead.err; exit 1; }
done
python - <<'PY'
import json
for l in open("gpurun_out/r4k/ab_aead.jsonl"):
    d = json.loads(l)
    print({k: v for k, v in d.items() if "ocb" in k or k in ("lib",)})
PY
