# round-end rehearsal: full GPU suite, smoke, bench defaults
R=$GRAFT_REPO_ROOT/gpurun_out/r37
mkdir -p $R
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $R/pytest.log 2>&1 || { tail -30 $R/pytest.log; exit 10; }
tail -1 $R/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $R/smoke.log 2>&1 || { tail -20 $R/smoke.log; exit 11; }
tail -1 $R/smoke.log
timeout -k 10 300 python -u bench.py > $R/bench.log 2>&1 || { tail -20 $R/bench.log; exit 12; }
tail -1 $R/bench.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $R/bench20.log 2>&1 || exit 13
tail -1 $R/bench20.log | cut -c1-200
timeout -k 10 300 python -u bench.py --gpus 2 --shared-gpu --steps 50 --warmup 10 > $R/bench_2rank.log 2>&1 || { tail -20 $R/bench_2rank.log; exit 14; }
tail -1 $R/bench_2rank.log | cut -c1-300
