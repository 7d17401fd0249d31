set -u
timeout -k 10 300 python -m pytest tests -m gpu -x -q 2>&1 | tail -5 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -3
