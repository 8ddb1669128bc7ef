cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=. && mkdir -p gpurun_out/sk
for m in 0 1 3; do timeout -k 10 300 python -u tools/conv_bench.py --kinds fwd,dgrad --small-k $m --only s0b0c1,s0b0c3,s0b1c1,s1b0c1,s1b0c3,s1b1c1,s2b0c1,s1b0proj > gpurun_out/sk/m$m.log 2>&1 || exit $?; done
