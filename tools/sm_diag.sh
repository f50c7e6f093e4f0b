set -o pipefail
export AZ_HIP_LIB=$PWD/alphazero-multi-game_amd/build_smdiag/libaz_hip.so
for v in ${VARIANTS:-1 2 3 4 5 6}; do echo "== variant $v"; AZ_SM_STAMPS=$v timeout -k 10 60 python tools/sm_stamps.py ${SMB:-256} | sed -n '2,4p;15,17p'; done
