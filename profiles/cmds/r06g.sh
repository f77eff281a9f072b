# r06g: bisect the min_1_norm N = 3 branch-and-bound status regression over the search's switches
set -o pipefail
export TMPDIR=/tmp
R=r06g
O=gpurun_out/${R}_l1_small.txt
TAG=default timeout -k 10 120 python profiles/diag_l1_small.py >> $O 2>&1
TAG=split1 HVP_SPLIT_LEVELS=1 timeout -k 10 120 python profiles/diag_l1_small.py >> $O 2>&1
TAG=lp_refill0 HVP_LP_REFILL=0 timeout -k 10 120 python profiles/diag_l1_small.py >> $O 2>&1
TAG=lp_root_refill0 HVP_LP_ROOT_REFILL=0 timeout -k 10 120 python profiles/diag_l1_small.py >> $O 2>&1
TAG=ipm HVP_L1_SIMPLEX=0 timeout -k 10 120 python profiles/diag_l1_small.py >> $O 2>&1
TAG=n5 timeout -k 10 120 python profiles/diag_l1_small.py l1_variant_n4_N5_qdu.npz >> $O 2>&1
TAG=n7 timeout -k 10 120 python profiles/diag_l1_small.py l1_variant_n3_N7.npz >> $O 2>&1
