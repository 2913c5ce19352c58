# round 4, session q: where the time goes now — phase ablations (-DBS_DIAG build,
# LDPC_DIAG_ABLATE: 1 no check phase, 2 no beta table, 4 no V->C pass, 8 no frame flags,
# 16 no iterations, 32 no LLR loads; timing only, results invalid) on C2 and C3
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_session.sh r4q ablate:C2:ab_libs/diag.so:0,1,2,4,8,16,32 ablate:C3:ab_libs/diag.so:0,1,2,4,8,16,32 || exit 1
