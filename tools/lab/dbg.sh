for d in 0 1 2 4 8 15; do echo "dbg=$d"; KW_DEC_DBG=$d timeout -k 10 100 python tools/kbench.py --only o_resid,fc2_resid,qkv_ln,o_plain,fc1_ln_gelu,xq_ln,lm_head || exit 1; done
