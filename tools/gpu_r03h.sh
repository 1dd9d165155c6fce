set -eo pipefail
timeout -k 10 300 python3 tools/debug/tail_mode.py 0 1073741824 0
timeout -k 10 300 python3 tools/debug/tail_mode.py 0 300 0
timeout -k 10 300 python3 tools/debug/tail_mode.py 1 1073741824 0
