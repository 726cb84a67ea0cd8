# same-box A/B: current build vs ab/libagx_base.so (tools/ab_lib.py), learn() time x3 each
set -o pipefail
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/learn_time.py 2>&1 | grep mean | sed "s/^/new:  /"
  AGX_LIB=ab/libagx_base.so timeout -k 10 120 python -u tools/learn_time.py 2>&1 | grep mean | sed "s/^/base: /"
done
