#!/bin/bash
# Runs GPU steps one after another on the gpurun box (step files under tools/steps/ are per-call
# scratch, kept out of git; what they produced is under profiles/): each line of the step file is
# "<seconds> <output file under gpurun_out/> <command...>". A step that fails ordinarily (exit 1-2,
# e.g. a failing test) does not stop the next one; a time limit (124/137), an abort (134) or a
# segmentation fault (139) ends the session there, as gpurun's rules require.
set -u
mkdir -p gpurun_out
while read -r secs out cmd; do
  [ -z "${secs:-}" ] && continue
  case "$secs" in \#*) continue ;; esac
  echo "[step] $cmd -> gpurun_out/$out ($(date +%T))"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$out" 2>&1
  rc=$?
  echo "[step] rc=$rc"
  case $rc in
    124|134|137|139) echo "[step] stopping after rc=$rc"; exit $rc ;;
  esac
done < "$1"
