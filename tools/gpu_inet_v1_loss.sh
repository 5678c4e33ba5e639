cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/iv1
for det in 0 1; do
DTF_DETERMINISTIC=$det timeout -k 10 300 python -u -m pytest -q -s --timeout 250 --timeout-method thread tests/test_gpu_imagenet_step.py -k "sizes3 or sizes4" > gpurun_out/iv1/det$det.log 2>&1
echo "det $det: $(grep -E 'loss rel' gpurun_out/iv1/det$det.log | tr '\n' ' ') $(tail -1 gpurun_out/iv1/det$det.log)"
done
