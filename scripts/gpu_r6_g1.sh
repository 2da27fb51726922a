cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_owned_operator_replay.py tests/test_gpu_exactness.py::test_c5_owner_unit_vs_oracle tests/test_gpu_exactness.py::test_c5_topk_benched_share_vs_oracle > gpurun_out/g1.log 2>&1
rc=$?
true
echo "tests rc=$rc bench rc=$?"
