cd "${GRAFT_REPO_ROOT}"
for rep in 1 2; do for v in wclk prio10 prio11 prio12; do
  echo "== $v"; GGRS_AMD_LIB=$PWD/ggrs_amd/var/lib_$v.so TPL=20 timeout -k 10 120 python3 -u tools/wave_clock.py 2>&1 | grep -E "^launch" | cut -c1-60 || exit 1
done; done
