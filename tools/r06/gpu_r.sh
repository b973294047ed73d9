# Round 6: check of the final tree after the small-job 16-bit committee tables.
OUT=gpurun_out/r06r bash tools/r06/gpu_f.sh
