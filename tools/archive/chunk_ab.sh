cd $GRAFT_REPO_ROOT
for rep in 1 2; do for ch in 0 32 64 128; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --opt stem_chunk=$ch > gpurun_out/ab_arm.log 2>&1 || { echo fail; tail -5 gpurun_out/ab_arm.log; exit 1; }
  python - $ch <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_arm.log").read().strip().splitlines()[-1])
st = d["stage_ms"]
groups = {"stem": ["conv1"], "112": ["conv4", "conv5", "conv6"], "56": ["conv7", "conv8", "conv9"],
          "28": ["conv10", "conv11", "conv12", "conv13"], "14": ["conv14", "conv15", "conv16", "conv17"],
          "tail": ["patch_embed", "transformer", "head"]}
g = {k: round(sum(st[s] for s in v), 3) for k, v in groups.items()}
print(f"chunk {sys.argv[1]:4s} {d['value']:9.1f} crops/s  {d['ms_per_step']:.3f} ms  {g}", flush=True)
PY
done; done
