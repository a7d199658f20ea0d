set -e
REPS=2 WORKLOAD=s3d bash tools/rvk_ab.sh "FAC_ND_IL=1" "FAC_ND_IL=0" "FAC_ND_IL=1 FAC_ND256_MIN=256"
REPS=2 bash tools/rvk_ab.sh "FAC_ND_IL=1" "FAC_ND_IL=1 FAC_ND256_MIN=256" "FAC_ND_IL=1 FAC_ND_TILE=2"
