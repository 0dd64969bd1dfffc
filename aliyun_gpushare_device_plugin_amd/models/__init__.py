"""Demo workloads run inside shared pods: the MFMA GEMM player and a Llama-3-8B-shaped model."""
