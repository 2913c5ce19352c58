# round 4, session o: the satisfied-wave alpha' skip on the one-chunk UCN instance (C3)
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_session.sh r4o ab:C3:ab_libs/uskip2.so,default:3 ab:C2:default,env=LDPC_BS_STAGGER=40,env=LDPC_BS_STAGGER=120:3 || exit 1
