# same-box A/B of learner variants: ab/libagx_<name>.so for each name given (plus the
# in-tree build as "tree"): phase stamps once, learn() time x2 interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.log
for n in "$@"; do
  lib=ab/libagx_$n.so; [ "$n" = tree ] && lib=agilerl_amd/lib/libagx.so
  echo "== $n stamps" >> gpurun_out/ab.log
  AGX_LIB=$lib timeout -k 10 120 python -u tools/learn_stamps.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab.log || exit 1
done
for i in 1 2; do
  for n in "$@"; do
    lib=ab/libagx_$n.so; [ "$n" = tree ] && lib=agilerl_amd/lib/libagx.so
    AGX_LIB=$lib timeout -k 10 120 python -u tools/learn_time.py 2>&1 | grep mean | sed "s/^/$n: /" >> gpurun_out/ab.log || exit 1
  done
done
cat gpurun_out/ab.log
