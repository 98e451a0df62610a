bash tools/gpu_r6.sh r6d tests "" "" && bash tools/gpu_r6_c4ab.sh r6d "0 3 4"
