# Round 6: check of the final tree after the small-job done flags.
OUT=gpurun_out/r06u bash tools/r06/gpu_f.sh
