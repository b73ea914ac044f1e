# Round 4 measurement pass on one box: GPU suite + smoke + default bench line (what the driver runs),
# the bench / rocprofv3 / PMC pass of every config, and the end-to-end / emulated-rank numbers.
set -e
R=$GRAFT_REPO_ROOT
OUT=${TAG:-r04g} bash $R/tools/gpu_suite.sh
OUT=${TAG:-r04g}_prof ENTRIES="ns:ns c3:c3 c5:c5 c2:c2 c4:c4 c1k:c1k" bash $R/tools/gpu_profile.sh
OUT=${TAG:-r04g}_e2e bash $R/tools/gpu_e2e.sh
echo done
