# Round 4: the whole GPU suite and smoke() on the tree as it stands.
OUT=gpurun_out/r04f
source tools/gpu_lib.sh
step gpu_tests 1050 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
echo ALL_DONE
