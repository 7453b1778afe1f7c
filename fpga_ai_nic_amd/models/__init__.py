"""fpga_ai_nic_amd.models."""
