for d in 0 1 2 4 7; do echo "FA_DBG=$d"; FA_DBG=$d timeout -k 10 100 python scripts/op_bench.py 2>&1 | grep FA; done
