bash tools/gpu_steps.sh \
 "breadth:::600:::python3 -u -m pytest tests/test_gpu_breadth.py -x -v --timeout 300 --timeout-method thread"
