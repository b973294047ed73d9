# Round 6: differential fuzz on the final tree (small jobs now on 16-bit committee combs with
# per-workgroup done flags; lone batches returning on the done word).
OUT=gpurun_out/r06v bash tools/r06/gpu_k.sh
