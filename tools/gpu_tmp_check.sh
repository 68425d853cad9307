set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/ab_libs.py --n 1024 --rounds 2 --compare reference=base:2 c_nochains=ab/lib_r6_c_nochains.so:2 c_norows=ab/lib_r6_c_norows.so:2 2>&1 | grep -v amdgpu.ids
