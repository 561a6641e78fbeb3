set -o pipefail
export TMPDIR=/tmp
for f in 0 64 128 256; do
  echo "== VISREPS_GRAM_FLUSH=$f"
  VISREPS_GRAM_FLUSH=$f DS=43264,186624,290400 timeout -k 10 200 python scripts/probe_gram.py 2>&1 | grep "N=" || exit 1
done
for f in 0 64 128; do
  echo "== accuracy VISREPS_GRAM_FLUSH=$f"
  VISREPS_GRAM_FLUSH=$f POINTS=conv1_post,conv2_pre,conv2_post,conv5_post,fc1_post timeout -k 10 300 python scripts/probe_gram_accuracy.py 2>&1 | grep "D=" || exit 1
done
