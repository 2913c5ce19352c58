# round 4, session i: C5 bsc instances after the position word (12-wave, CPL 3 mixed, uniform)
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_session.sh r4i ab:C5:default,env=LDPC_BSC_INST=3,env=LDPC_BSC_INST=2,env=LDPC_BSC_INST=0:2 || exit 1
