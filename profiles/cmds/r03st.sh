# r03s + r03t in one call (the pool is congested): heavy-platoon incumbent experiment, then the
# re-profile of HEAD and the default bench
set -o pipefail
bash profiles/cmds/r03s.sh || exit 1
bash profiles/cmds/r03t.sh || exit 2
