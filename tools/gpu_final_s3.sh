# Final pass of round 3's last session: GPU suite, smoke(), the default bench line, and the NS /
# C3 / C5 profile pass (bench, rocprofv3 --kernel-trace --stats, PMC FETCH/WRITE passes).
set -e
R=$GRAFT_REPO_ROOT
OUT=final_s3 bash $R/tools/gpu_suite.sh
OUT=final_s3_prof ENTRIES="ns:ns c3:c3 c5:c5" bash $R/tools/gpu_profile.sh
echo done
