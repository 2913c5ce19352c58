# round 4, session d: A/B of this round's bit-sliced changes, the flood and e2e profiles
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_session.sh r4d ab:C4:ab_libs/gbl1.so,ab_libs/bkpf0.so,default,env=LDPC_BS_INST=7:2 ablate:C4:ab_libs/diag.so:0,1,2,4,8,16,32 ab:C3:ab_libs/bkpf0.so,ab_libs/bkpf2.so,default:2 ab:C2:ab_libs/head.so,ab_libs/bkpf0.so,ab_libs/bkpf2.so,default:2 || exit 1
K=flood CFG=C2 TAG=r4 B=1048576 bash tools/profile.sh || exit 1
K=auto CFG=C2 TAG=e2e PROF_EXTRA=--e2e bash tools/profile.sh || exit 1
