export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/smoke.log; exit $rc
