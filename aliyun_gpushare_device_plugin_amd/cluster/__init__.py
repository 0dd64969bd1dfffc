"""Cluster state (L2): apiserver client, node-status patch, pod watch cache, kubelet client."""
