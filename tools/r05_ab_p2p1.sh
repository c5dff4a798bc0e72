cd "${GRAFT_REPO_ROOT}"
for rep in 1 2; do
 for v in base cur; do
  lib=$PWD/ggrs_amd/libggrs_amd.so; [ $v = base ] && lib=$PWD/ggrs_amd/var/lib_base.so
  echo "== $v"
  GGRS_AMD_LIB=$lib LINES="p2p1 p2p1_131k p2p1_1m" bash tools/r05_lines.sh || exit 1
 done
done
