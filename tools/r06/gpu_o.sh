# Round 6: check of the final tree after the done-word default (suite, smoke, bench line).
OUT=gpurun_out/r06o bash tools/r06/gpu_f.sh
