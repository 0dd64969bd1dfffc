"""How long a process takes to die after SIGTERM (default action), by what it did on the GPU:
nothing, HIP initialised, a stream and a kernel, 6 GiB held. Timed from the signal to the
parent's blocking waitpid return (the process is gone). One JSON line per case and trial."""
import json
import signal
import subprocess
import sys
import time

CASES = {
    "python_only": "import sys, time; print('ready', flush=True); time.sleep(600)",
    "torch_imported": "import sys, time, torch; print('ready', flush=True); time.sleep(600)",
    "hip_init": "import sys, time, torch; torch.cuda.init(); print('ready', flush=True); time.sleep(600)",
    "first_kernel": ("import sys, time, torch; x = torch.ones(1 << 20, device='cuda'); x.add_(1); "
                     "torch.cuda.synchronize(); print('ready', flush=True); time.sleep(600)"),
    "held_6gib": ("import sys, time, torch; x = torch.ones(6 << 29, dtype=torch.bfloat16, device='cuda'); "
                  "torch.cuda.synchronize(); print('ready', flush=True); time.sleep(600)"),
}

for trial in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    for name, code in CASES.items():
        p = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True)
        assert p.stdout.readline().strip() == "ready"
        time.sleep(0.3)
        t0 = time.perf_counter()
        p.send_signal(signal.SIGTERM)
        p.wait()                                   # blocking waitpid: no polling granularity
        print(json.dumps({"case": name, "trial": trial, "exit_ms": round((time.perf_counter() - t0) * 1e3, 2)}),
              flush=True)
        time.sleep(1.0)                            # the previous teardown's deferred work is done
