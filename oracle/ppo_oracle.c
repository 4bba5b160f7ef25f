/* ORACLE — test infrastructure only (placeholder, filled in with the PPO restatement). */
int oracle_ppo_version(void) { return 1; }
