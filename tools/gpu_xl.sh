# Whole-line f64 stores in the product (fused row-major groups at KG <= 3): GPU suite, then the
# bench + rocprof + PMC pass of C3 / C5 / NS.
set -e
R=$GRAFT_REPO_ROOT
OUT=xl bash $R/tools/gpu_suite.sh
OUT=xl_prof ENTRIES="c3:c3 c5:c5 ns:ns" bash $R/tools/gpu_profile.sh
echo done
