"""Golden-vector case table (plain data; shared by make_golden.py and the tests).

Each case is a tiny instance of one BASELINE.json config family. Shapes follow the reference's
own configs (configs/model/*.yaml, configs/experiment/*.yaml) scaled down so the CPU oracle
finishes in well under a second.
"""

CASES = {
    # BaseVAE with attention at a non-mid level (attn_resolutions=[16] at 16x16 -> 256 tokens),
    # GroupNorm with 1 and 2 channels per group, Downsample 16->8 and Upsample 8->16.
    "base_attn": dict(
        cls="BaseVAE",
        kwargs=dict(input_channels=3, latent_dim=8, hidden_channels=32, ch_mult=[1, 2],
                    num_res_blocks=1, attn_resolutions=[16], dropout=0.0, resolution=16),
        batch=2, cond="none",
        loss=dict(type="vae", recon_loss_type="mse", kl_weight=1.0, recon_weight=1.0),
        optimizer=dict(type="adamw", lr=2e-4, weight_decay=1e-4, betas=[0.9, 0.999]),
        clip=1.0,
    ),
    # Config 2 family (path_beta_vae at 28x28x3, ch_mult (1,2,4)): odd spatial sizes 28->14->7.
    "beta_c2": dict(
        cls="BetaVAE",
        kwargs=dict(input_channels=3, latent_dim=16, hidden_channels=32, ch_mult=[1, 2, 4],
                    num_res_blocks=2, attn_resolutions=[], dropout=0.0, resolution=28, beta=6.0),
        batch=3, cond="none",
        loss=dict(type="vae", recon_loss_type="mse", kl_weight=6.0, recon_weight=1.0),
        optimizer=dict(type="adamw", lr=1e-4, weight_decay=1e-4, betas=[0.9, 0.999]),
        clip=1.0,
    ),
    # Config 1 family (chest_base_vae, 1-channel input).
    "base_c1": dict(
        cls="BaseVAE",
        kwargs=dict(input_channels=1, latent_dim=16, hidden_channels=32, ch_mult=[1, 2, 4],
                    num_res_blocks=1, attn_resolutions=[], dropout=0.0, resolution=28),
        batch=2, cond="none",
        loss=dict(type="vae", recon_loss_type="mse", kl_weight=1.0, recon_weight=1.0),
        optimizer=dict(type="adamw", lr=2e-4, weight_decay=1e-4, betas=[0.9, 0.999]),
        clip=1.0,
    ),
    # Config 4 family (multi_modal_cvae: ConditionalVAE concat, 12-way one-hot, ch_mult (1,2,4,8),
    # attention at 16) at 32x32 so that 16x16 attention sits at level 1.
    "cvae_c4": dict(
        cls="ConditionalVAE",
        kwargs=dict(input_channels=3, latent_dim=8, hidden_channels=16, ch_mult=[1, 2, 4, 8],
                    num_res_blocks=1, attn_resolutions=[16], dropout=0.0, resolution=32,
                    condition_method="concat"),
        batch=3, cond="onehot",
        loss=dict(type="vae", recon_loss_type="mse", kl_weight=1.0, recon_weight=1.0),
        optimizer=dict(type="adamw", lr=1e-4, weight_decay=1e-5, betas=[0.5, 0.999]),
        clip=1.0,
    ),
    # Config 3 family (disentangled_multi_modal_cvae_quick), dropout forced to 0 for parity,
    # mixed gray/colour batch with an out-of-range modality index (7 -> clamped to 4).
    "dis_c3": dict(
        cls="DisentangledConditionalVAE",
        kwargs=dict(num_modalities=5, shared_latent_dim=8, modality_latent_dim=8,
                    hidden_channels=32, ch_mult=[1, 2, 4], num_res_blocks=1, attn_resolutions=[],
                    dropout=0.0, resolution=28, modality_separation_weight=0.1,
                    contrastive_weight=0.05),
        batch=8, cond="idx", idx=[0, 1, 2, 3, 4, 7, 1, 0],
        loss=dict(type="disentangled_vae", recon_loss_type="mse", kl_weight=1.0,
                  recon_weight=1.0, separation_weight=0.1, contrastive_weight=0.05),
        optimizer=dict(type="adam", lr=5e-4, weight_decay=0.0, betas=[0.9, 0.999]),
        clip=0.5,
    ),
    # ---- full BASELINE architectures at small batch (the production fast paths: 256x256 GEMM tiles,
    # GroupNorm statistics / backward fused into the GEMM epilogues (H*W % 32 == 0, C/G % 4 == 0),
    # sub-pixel Upsample at >= 512 channels, many-split wgrad, 1024/2048-channel attention).
    # Config 4 exactly (configs/experiment/multi_modal_cvae.yaml + model.resolution=64, loss vae,
    # configs/training/advanced.yaml optimizer): 927 M parameters.
    "cvae_c4_full": dict(
        cls="ConditionalVAE",
        kwargs=dict(input_channels=3, latent_dim=256, hidden_channels=256, ch_mult=[1, 2, 4, 8],
                    num_res_blocks=2, attn_resolutions=[16], dropout=0.0, resolution=64,
                    condition_method="concat"),
        batch=2, cond="onehot", full=True,
        loss=dict(type="vae", recon_loss_type="mse", kl_weight=1.0, recon_weight=1.0),
        optimizer=dict(type="adamw", lr=1e-4, weight_decay=1e-5, betas=[0.5, 0.999]),
        clip=1.0,
    ),
    # Config 2 exactly (path_beta_vae, 3-level ch_mult at 28x28x3; mid attention only).
    "beta_c2_full": dict(
        cls="BetaVAE",
        kwargs=dict(input_channels=3, latent_dim=128, hidden_channels=128, ch_mult=[1, 2, 4],
                    num_res_blocks=2, attn_resolutions=[16], dropout=0.0, resolution=28, beta=6.0),
        batch=2, cond="none", full=True,
        loss=dict(type="vae", recon_loss_type="mse", kl_weight=6.0, recon_weight=1.0),
        optimizer=dict(type="adamw", lr=1e-4, weight_decay=1e-4, betas=[0.9, 0.999]),
        clip=1.0,
    ),
    # Config 1 exactly (chest_base_vae at 28x28x1 with the 3-level ch_mult, hidden 128, z 256, two ResnetBlocks per
    # level; configs/experiment/chest_base_vae.yaml, BASELINE config 1).
    "base_c1_full": dict(
        cls="BaseVAE",
        kwargs=dict(input_channels=1, latent_dim=256, hidden_channels=128, ch_mult=[1, 2, 4],
                    num_res_blocks=2, attn_resolutions=[16], dropout=0.0, resolution=28),
        batch=2, cond="none", full=True,
        loss=dict(type="vae", recon_loss_type="mse", kl_weight=1.0, recon_weight=1.0),
        optimizer=dict(type="adamw", lr=2e-4, weight_decay=1e-4, betas=[0.9, 0.999]),
        clip=1.0,
    ),
    # Config 3 architecture (disentangled_multi_modal_cvae_quick) at B=16: every modality, repeated
    # modalities, and out-of-range ids 7, 9 and 17 (routing clamps them to 4; the separation loss keeps
    # each as its own centroid, so ids >= 16 must work too).
    "dis_c3_b16": dict(
        cls="DisentangledConditionalVAE",
        kwargs=dict(num_modalities=5, shared_latent_dim=8, modality_latent_dim=8,
                    hidden_channels=32, ch_mult=[1, 2, 4], num_res_blocks=1, attn_resolutions=[],
                    dropout=0.0, resolution=28, modality_separation_weight=0.1,
                    contrastive_weight=0.05),
        batch=16, cond="idx", idx=[0, 1, 2, 3, 4, 7, 1, 0, 17, 3, 2, 4, 4, 9, 1, 0],
        loss=dict(type="disentangled_vae", recon_loss_type="mse", kl_weight=1.0,
                  recon_weight=1.0, separation_weight=0.1, contrastive_weight=0.05),
        optimizer=dict(type="adam", lr=5e-4, weight_decay=0.0, betas=[0.9, 0.999]),
        clip=0.5,
    ),
}

MODALITY_CHANNELS = {0: 1, 1: 3, 2: 3, 3: 1, 4: 3}

# Parameters whose full gradient / updated value is stored in the fixture (others: sum + sumsq).
FULL_GRADS = {
    "base_attn": ["encoder.conv_in.weight", "encoder.down.0.attn.0.q.weight",
                  "decoder.up.0.block.1.norm1.weight", "decoder.conv_out.bias",
                  "encoder.down.0.downsample.conv.weight", "decoder.up.1.upsample.conv.bias"],
    "beta_c2": ["encoder.conv_out.weight", "decoder.mid.attn_1.proj_out.weight",
                "encoder.down.1.block.0.nin_shortcut.weight"],
    "base_c1": ["encoder.conv_in.weight", "decoder.conv_out.weight"],
    "cvae_c4": ["condition_proj.0.weight", "condition_proj.0.bias", "encoder.conv_in.weight",
                "encoder.down.1.attn.0.k.weight"],
    "dis_c3": ["modality_input_projectors.0.weight", "modality_output_projectors.3.weight",
               "modality_decoders.4.0.weight", "modality_decoders.1.2.bias",
               "encoder.conv_in.weight"],
    "cvae_c4_full": ["condition_proj.0.bias", "encoder.conv_in.weight", "decoder.conv_out.weight",
                     "decoder.conv_out.bias", "encoder.mid.attn_1.norm.weight", "decoder.up.3.block.0.norm1.bias",
                     "encoder.norm_out.weight"],
    "beta_c2_full": ["encoder.conv_in.weight", "decoder.conv_out.weight", "decoder.mid.attn_1.proj_out.bias",
                     "encoder.down.1.block.0.nin_shortcut.weight", "decoder.up.0.block.2.norm2.weight"],
    "base_c1_full": ["encoder.conv_in.weight", "decoder.conv_out.weight", "decoder.mid.attn_1.v.bias",
                     "encoder.down.2.block.1.norm2.bias", "decoder.up.1.block.2.conv1.bias"],
    "dis_c3_b16": ["modality_input_projectors.0.weight", "modality_output_projectors.3.weight",
                   "modality_decoders.4.0.weight", "modality_decoders.1.2.bias", "modality_decoders.2.2.weight",
                   "encoder.conv_in.weight"],
}
