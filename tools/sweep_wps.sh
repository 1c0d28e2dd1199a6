export DABGPU_ACS_WPS=5
bash tools/gpu_steps.sh t5 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "pipeline" || exit 1
for w in 0 3 4 5 6 8; do
  DABGPU_ACS_WPS=$w bash tools/gpu_steps.sh w$w 200 python bench.py --no-cpu-baseline || exit 1
done
