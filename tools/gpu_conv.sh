cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 python tools/debug_conv.py > gpurun_out/conv.log 2>&1 && N2V2R_RR_CLUSTER=1e-3 timeout -k 10 120 python tools/debug_conv.py >> gpurun_out/conv.log 2>&1
