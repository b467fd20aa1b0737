export TAG=r4b
bash tools/gpu_round.sh results && bash tools/gpu_round.sh profile && bash tools/gpu_round.sh pmc && \
AB_CFGS="base: small0:LPC_BUDGET_SMALL=0 small48:LPC_BUDGET_SMALL=48" bash tools/gpu_round.sh ab
