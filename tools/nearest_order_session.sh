set -u
ROUNDS=1 bash tools/ab_session.sh ab_near_dragon --steps 600 --warmup 60 &&
ROUNDS=1 bash tools/ab_session.sh ab_near_happy --scene happy --steps 600 --warmup 60 &&
ROUNDS=1 bash tools/ab_session.sh ab_near_happy4k --scene happy --width 3840 --height 2160 --steps 300 --warmup 30 &&
ROUNDS=1 bash tools/ab_session.sh ab_near_c3 --width 960 --height 540 --steps 600 --warmup 60
