cd $GRAFT_REPO_ROOT
tools/gpu_run.sh "gpu_tests:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit 1
tools/variants.sh pre_l2e base
