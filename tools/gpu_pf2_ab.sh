set -e
export TMPDIR=/tmp
bash tools/ab_env.sh r03_pf2 split:- pf2:pf2 npf2:npf2 npf2w7:npf2w7
