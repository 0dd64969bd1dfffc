"""High-fidelity fakes for CPU-only end-to-end runs: apiserver, kubelet, extender, cluster."""
