cd $GRAFT_REPO_ROOT
timeout -k 10 120 python scripts/pub_time.py 4096
