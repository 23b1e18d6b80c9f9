cd "$GRAFT_REPO_ROOT" || exit 3
MESH_TIME=1 timeout -k 10 120 python tools/mesh_debug.py 4096 | grep "^time" || exit 1
./tools/gpu_mesh.sh
