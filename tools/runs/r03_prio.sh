# Stream-priority A/B of the two bench engines (round 3, not kept): a variant
# build whose engine_create read SRTP_PRIO_ENGINES ("hl": engine 0 high, 1 low).
cd "${GRAFT_REPO_ROOT}"
export SRTP_MI355X_LIB=$PWD/libjitsi_amd/variants/libsrtp_prio.so  # built from an engine.cpp with the SRTP_PRIO_ENGINES knob
O=gpurun_out/r03_prio; mkdir -p $O
for rep in 1 2; do
  for P in none hl lh; do
    if [ $P = none ]; then unset SRTP_PRIO_ENGINES; else export SRTP_PRIO_ENGINES=$P; fi
    timeout -k 10 120 python bench.py --steps 30 --no-cpu --no-e2e --no-dispatch > $O/b_$P.log 2>&1 || { echo "bench failed $P"; tail -5 $O/b_$P.log; exit 1; }
    python -c "import json; l=[x for x in open('$O/b_$P.log') if x.startswith('{')][-1]; j=json.loads(l); print('$P', round(j['value']/1e6,1), j['ms_per_step'])"
  done
done
