# round 4, session f: C4 A/B — C->V kept in registers for more edges on the multi-chunk
# instances (BS_KEEP_MC), the first-generation start spread
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_session.sh r4f ab:C4:ab_libs/keep6.so,ab_libs/keep7.so,default,env=LDPC_BS_STAGGER=50,env=LDPC_BS_STAGGER=200,env=LDPC_BS_STAGGER=0:2 || exit 1
