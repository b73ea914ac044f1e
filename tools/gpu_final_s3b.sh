# Last pass of the session with the final kernels (whole-line f64 stores in C3's instance): GPU
# suite, smoke(), default bench, and the bench / rocprofv3 / PMC pass of every config.
set -e
R=$GRAFT_REPO_ROOT
OUT=final_s3b bash $R/tools/gpu_suite.sh
OUT=final_s3b_prof ENTRIES="ns:ns c3:c3 c5:c5 c2:c2 c4:c4 c1k:c1k" bash $R/tools/gpu_profile.sh
echo done
