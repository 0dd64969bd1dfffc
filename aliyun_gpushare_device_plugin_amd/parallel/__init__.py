"""Multi-GPU concerns: xGMI topology export, TP-group placement, RCCL validation demo."""
