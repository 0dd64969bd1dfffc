"""Device layer: SMI binding (L0), fake-device model (L1), health monitor."""
