# Run several GPU scripts in one call; a later one starts only if the earlier ones ended normally or
# with an ordinary failure (not a time limit, abort or crash: 124 / 134 / 137 / 139 end the call).
for s in "$@"; do
  bash "$s"
  rc=$?
  echo "[chain] $s -> $rc"
  case $rc in 124|134|137|139) exit $rc ;; esac
done
