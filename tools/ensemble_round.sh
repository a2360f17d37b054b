mkdir -p gpurun_out/ens5
timeout -k 10 200 python -u -m pytest tests/test_ensemble.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ens5/pytest.txt 2>&1 || { tail -30 gpurun_out/ens5/pytest.txt; exit 1; }
tail -1 gpurun_out/ens5/pytest.txt
for v in "--tpe 2" "--tpe 1" "--tpe 2 --spg 100" "--tpe 1 --spg 100" "--tpe 2 --steps 600 --spg 100"; do
  echo "== $v"; timeout -k 10 120 python -u tools/ensemble_probe.py --members 1,2,3 $v > gpurun_out/ens5/p.txt 2>&1 || exit 1
  grep "^[123] " gpurun_out/ens5/p.txt | cut -c1-150 | tee -a gpurun_out/ens5/probe_summary.txt
done
for m in 1 2; do timeout -k 10 120 python -u -m stsphere ensemble sharding-the-sphere-fall-2025-jax-devlab-examples_amd/configs/reference_6dev.yaml --members $m --nsteps 600 > gpurun_out/ens5/c96_m$m.txt 2>&1 || exit 1; tail -1 gpurun_out/ens5/c96_m$m.txt; done
