set -o pipefail
D=gpurun_out/r6w
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -s tests/test_hbm_broker.py -k "zeros or retiring or released_arena or scrub" > $D/tests.log 2>&1 \
 && timeout -k 10 120 python -u tools/diag/scrub_pmc_driver.py > $D/plain.jsonl 2>&1 \
 && timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $D/kt -o scrub -- python -u tools/diag/scrub_pmc_driver.py > $D/kt.log 2>&1
