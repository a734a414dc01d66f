# round 6: kernel trace + counter passes of the bench (the headline kernel) on the shipped library
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/profile_box.sh ${1:-r6prof} && python3 tools/pmc_traffic.py gpurun_out/${1:-r6prof} gpurun_out/${1:-r6prof}/k_djn_pmd_pmc.json --win 23 --n 1000000 --kernel k_djn_pmd
