# round 4: the four bench configs with the mix ceiling (no CPU leg)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4i; mkdir -p $O
for c in 20:3 10:3dec 20:3loss1; do
  timeout -k 10 300 python bench.py --config $c --no-cpu > $O/bench_${c/:/}.json 2> $O/bench_${c/:/}.err || { cat $O/bench_${c/:/}.err; exit 1; }
done
timeout -k 10 300 python bench.py --config 200:55 --no-cpu --steps 5 > $O/bench_20055.json 2> $O/bench_20055.err || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4i/bench_*.json")):
    d = json.load(open(f)); r = d["roofline"]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d.get("encode_ms"), d["decode_ms"], "frac", r.get("frac"), "read_ceil", r.get("read_ceiling"), r.get("frac_of_ceiling"), "mix", r.get("mix_ceiling"), r.get("frac_of_mix_ceiling"), r.get("decode_frac"))
PY
