# Round 4 closing pass, part 2: the profile pass of C2, C4, C1k and the end-to-end / emulated-rank
# numbers (tools/gpu_e2e.sh).
set -e
R=$GRAFT_REPO_ROOT
OUT=r04z_prof ENTRIES="c2:c2 c4:c4 c1k:c1k" bash $R/tools/gpu_profile.sh
OUT=r04z_e2e bash $R/tools/gpu_e2e.sh
echo done
