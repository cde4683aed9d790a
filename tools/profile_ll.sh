set -o pipefail
for a in ll oneshot; do for n in 2 8; do
  DIRECT_TAG=${a}_n$n DIRECT_N=$n DIRECT_KIB="32" DIRECT_ALGOS=$a bash tools/profile_direct.sh || exit 3
done; done
echo all done
