cd "$GRAFT_REPO_ROOT"
L=optical-flow-using-dense-inverse-search_amd/disflow/libdis_hip.so
bash tools/gpu/tests.sh tests/test_cpp_facade.py tests/test_gpu_parity.py && timeout -k 10 600 python3 tools/ab.py $L $L:variant=5 $L:fma=1 $L:fma=1,variant=5 --rounds 6 --steps 10
