bash tools/r3_glue.sh g3 tests/test_gpu_kernels.py tests/test_gpu_bench_geometry.py tests/test_gpu_bf16_dma.py && bash tools/r3_pmc_evidence.sh pmcev
