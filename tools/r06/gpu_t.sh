# Round 6: the small-job done flags again, with early-released jobs kept off the free list
# until their launch has finished (DevPool::retiring).
OUT=gpurun_out/r06t bash tools/r06/gpu_s.sh
