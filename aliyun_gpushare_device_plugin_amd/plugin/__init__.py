"""Device-plugin layer (L3/L4): gRPC server, lifecycle manager, watchers."""
