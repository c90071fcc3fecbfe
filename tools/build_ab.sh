# builds libgmat_hip.so of a commit into ab/lib_<name>.so (in-tree, so that it travels to the GPU box;
# select it with GMAT_HIP_LIB=ab/lib_<name>.so in tools/env_ab.sh arms): bash tools/build_ab.sh REV NAME
set -e
rev=$1; name=$2
wt=/tmp/gmat_wt_$name
rm -rf $wt; git worktree prune
git worktree add -f --detach $wt $rev > /dev/null
mkdir -p ab
make -s -j8 -C $wt/gmat_amd/csrc OUT=$(pwd)/ab/lib_$name.so
git worktree remove --force $wt
echo "ab/lib_$name.so from $(git rev-parse --short $rev)"
