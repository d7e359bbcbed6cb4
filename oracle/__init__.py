"""TEST INFRASTRUCTURE ONLY: the CPU oracle (see gs_oracle.h). Product code never imports this."""
