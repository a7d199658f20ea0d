#!/bin/bash
# Same-box A/B of builds of the library, alternating arms, 2 rounds.
# Arms: $AB_LIBS (space-separated .so paths, "tree" = the in-tree build),
# default "fac_fake_amd/libfac_cvit_base.so tree" (tools/build_base_lib.sh).
# Extra args go to bench.py.
mkdir -p gpurun_out
ARMS=${AB_LIBS:-"$(pwd)/fac_fake_amd/libfac_cvit_base.so tree"}
for rep in 1 2; do
  for arm in $ARMS; do
    if [ $arm = tree ]; then unset FAC_CVIT_LIB; else export FAC_CVIT_LIB=$(realpath $arm); fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/ab_arm.log 2>&1 || { echo "arm $arm failed"; tail -5 gpurun_out/ab_arm.log; exit 1; }
    python - "$(basename $arm)" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_arm.log").read().strip().splitlines()[-1])
st = d["stage_ms"]
groups = {"stem": ["conv1"], "112": ["conv4", "conv5", "conv6"], "56": ["conv7", "conv8", "conv9"],
          "28": ["conv10", "conv11", "conv12", "conv13"], "14": ["conv14", "conv15", "conv16", "conv17"],
          "tail": ["patch_embed", "transformer", "head"]}
g = {k: round(sum(st[s] for s in v), 3) for k, v in groups.items()}
print(f"{sys.argv[1][:22]:22s} {d['value']:9.1f} crops/s  {d['ms_per_step']:.3f} ms  {g}", flush=True)
PY
  done
done
