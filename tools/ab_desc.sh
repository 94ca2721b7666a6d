# A/B of the descriptor kernel variant (1: k_desc_kp, 4 waves per keypoint; 0: k_desc, one wave).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for m in 1 0; do echo desc_mode=$m; ORBHIP_DESC_MODE=$m timeout -k 10 200 python bench.py --no-cpu --no-extra 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], c['sequential_frames_per_s'], c['sixteen_cameras_frame_by_frame_frames_per_s'], c['host_submit_ms_per_frame'])"; done
