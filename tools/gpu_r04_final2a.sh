# Round 4 closing pass, part 1: GPU suite + smoke + default bench line, then the bench / rocprofv3 /
# PMC pass of NS, C3, C5 with the final tree.
set -e
R=$GRAFT_REPO_ROOT
OUT=r04z bash $R/tools/gpu_suite.sh
OUT=r04z_prof ENTRIES="ns:ns c3:c3 c5:c5" bash $R/tools/gpu_profile.sh
echo done
