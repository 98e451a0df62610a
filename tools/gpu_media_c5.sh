bash tools/gpu_media.sh && bash tools/gpu_c5.sh 64 2
