# A/B two builds of the extension on the SAME GPU box: tools/ab_so.sh "<cmd>" [variants...]
# (variants are ab/<name>.so copies of imitation_amd/_C*.so; each runs <cmd> once, alternating twice)
set -o pipefail
cd $GRAFT_REPO_ROOT
SO=$(ls imitation_amd/_C.cpython-*.so)
CMD=$1; shift
cp $SO /tmp/orig.so
for rep in 1 2; do
  for v in "$@"; do
    cp ab/$v.so $SO
    echo "== $v (rep $rep)"
    timeout -k 10 300 bash -c "$CMD" || { cp /tmp/orig.so $SO; exit 1; }
  done
done
cp /tmp/orig.so $SO
