"""MI355X-native GP-MPC solve path (drop-in for amacati/gp-mpc's ``gpmpc`` package)."""
