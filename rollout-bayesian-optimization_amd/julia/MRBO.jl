# MRBO.jl -- Julia binding of libmrbo.so (include/mrbo.h) for the reference package.
#
# The reference is not a package: rollout_bayesian_optimization.jl:1-30 `include`s its files into
# `Main`, so its types (Surrogate, Trajectory, TrajectoryParameters, ...) and generic functions
# (simulate_trajectory_mc, simulate_trajectory_ghq, the get_* accessors) are bindings of `Main`.
# This module therefore takes every reference name it uses from `Main` explicitly, and
# `import`s the two generic functions it adds methods to, so that the methods below extend the
# reference's own `simulate_trajectory_mc` (rollout.jl:279-340) and `simulate_trajectory_ghq`
# (rollout.jl:409-467) rather than defining new functions:
#
#     include("rollout_bayesian_optimization.jl")
#     include("path/to/rollout-bayesian-optimization_amd/julia/MRBO.jl"); using .MRBO
#     eto = simulate_trajectory_mc(T, tp, MrboBackend(0); inner_solve_xstarts=..., resolutions=..., ...)
#
# The GPU methods keep the reference's keyword contract: caller-owned containers overwritten in
# place, an ExpectedTrajectoryOutput returned, T.x0 set from tp (T.θ kept, Q12), an exception on a
# failed trajectory.  The trailing `MrboBackend` positional argument selects them; it is not an
# AbstractObservable, so the reference's observable overload (rollout.jl:342) is not ambiguous.
#
# julia is not installed in this image, so the file is never executed here.  What can be checked
# without julia is checked by tests/test_julia_binding.py: the struct mirrors against the C
# structs of include/mrbo.h (field order, types, offsets), every ccall against its C prototype,
# and every reference name used here against the names this module brings into scope from Main.
module MRBO

# the reference's generic functions this module adds methods to (must be `import`ed to extend)
import Main: simulate_trajectory_mc, simulate_trajectory_ghq, stochastic_solve
# the reference's types, constructors and accessors used below (Main-level bindings)
using Main: Surrogate, Trajectory, TrajectoryParameters, ExpectedTrajectoryOutput,
            StochasticGradientAscent, StandardSGA, Adam, ExperimentSetup, get_starts,
            Matern52, Matern32, Matern12, SquaredExponential, Periodic,
            get_observed, get_active_covariates, get_active_cholesky, get_active_coefficients,
            get_active_observations, get_observations, get_kernel, get_decision_rule, get_name,
            get_spatial_bounds, get_starting_point, get_base_surrogate, set_start!
import Distributions

export MrboBackend, MrboPlan, mrbo_multistart_base_solve!, mrbo_log_likelihood, mrbo_release_plans!

const libmrbo = joinpath(@__DIR__, "..", "mrbo", "libmrbo.so")
const MRBO_FLAG_HOST_POINTERS = UInt32(1)
const MRBO_FLAG_NO_GRADIENT = UInt32(2)

# mirrors mrbo_surrogate_t (include/mrbo.h; Julia isbits structs use the C layout)
struct MrboSurrogateC
    d::Int32
    N::Int32
    kernel::Int32
    lengthscale::Float64
    sigma_n2::Float64
    fmini::Float64
    X::Ptr{Float64}
    L::Ptr{Float64}
    ldL::Int32
    c::Ptr{Float64}
    y::Ptr{Float64}
    period::Float64      # Periodic θ[2]
end

# mirrors mrbo_params_t
struct MrboParamsC
    h::Int32
    M::Int32
    R::Int32
    nstarts::Int32
    rule::Int32
    theta::Float64
    lbs::Ptr{Float64}
    ubs::Ptr{Float64}
    max_iters::Int32
    max_ls::Int32
    x_tol::Float64
    f_tol::Float64
    g_tol::Float64
    htol::Float64
    sigma_tol::Float64
    seed::UInt64
    sample_offset::Int32
    samples_total::Int32
    cost::Int32          # mrbo_cost_t: NonUniformCost weighting of the inner-solve rule (0 = none)
    cost_c0::Float64
    cost_w::Ptr{Float64}
end

# mirrors mrbo_solve_opts_t (the outer ascent of mrbo_stochastic_solve)
struct MrboSolveOptsC
    optimizer::Int32     # 0 StandardSGA, 1 Adam
    iterations::Int32
    eta::Float64
    beta1::Float64
    beta2::Float64
    eps::Float64
    sample_size::Float64 # eswavs sample size (0 → the plan's M = tp.mc_iters)
end

mrbo_solve_opts(o::StandardSGA, iterations::Int) = MrboSolveOptsC(Int32(0), Int32(iterations), o.η, 0.9, 0.999, 1e-8, 0.0)
mrbo_solve_opts(o::Adam, iterations::Int) = MrboSolveOptsC(Int32(1), Int32(iterations), o.η, o.β1, o.β2, o.ε, 0.0)

struct MrboBackend
    device::Int
end
MrboBackend() = MrboBackend(0)

mutable struct MrboPlan
    handle::Ptr{Cvoid}
    d::Int
    M::Int
    R::Int
    h::Int
end

mrbo_kernel_id(ψ) = ψ.constructor === Matern52 ? Int32(0) : ψ.constructor === Matern32 ? Int32(1) :
                    ψ.constructor === Matern12 ? Int32(2) : ψ.constructor === SquaredExponential ? Int32(3) :
                    ψ.constructor === Periodic ? Int32(4) : error("kernel not compiled into libmrbo")
mrbo_kernel_period(ψ) = ψ.constructor === Periodic ? Float64(ψ.θ[2]) : 1.0

function mrbo_check(rc)
    rc == 0 && return nothing
    msg = unsafe_string(ccall((:mrbo_last_error, libmrbo), Cstring, ()))
    error("libmrbo error $rc: $msg")
end

mrbo_rule_id(g) = get_name(g) == "EI" ? Int32(0) : get_name(g) == "POI" ? Int32(1) :
                  get_name(g) == "LCB" ? Int32(2) : error("decision rule not compiled into libmrbo")

# The device state of simulate_trajectory_mc's setup: FantasySurrogate(s, h) over the base
# surrogate (radial_basis_surrogates.jl:345-381) + TrajectoryParameters (trajectory.jl:43-94),
# for R restart points per launch.  The caller owns the returned plan and must release it with
# mrbo_plan_destroy!; the rollout methods below take theirs from the plan cache instead.
function MrboPlan(s::Surrogate, tp::TrajectoryParameters, θ::Vector{Float64}, nstarts::Int;
                  device::Int = 0, max_iters = 50, max_ls = 20, seed = 1906, M::Int = tp.mc_iters, R::Int = 1)
    N = get_observed(s)
    X = Matrix{Float64}(get_active_covariates(s))
    L = Matrix{Float64}(get_active_cholesky(s))
    c = Vector{Float64}(get_active_coefficients(s))
    y = Vector{Float64}(get_active_observations(s))
    fmini = minimum(get_observations(s))                 # over the capacity buffer (Q3)
    lbs, ubs = get_spatial_bounds(tp)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve X L c y lbs ubs begin
        sd = MrboSurrogateC(Int32(size(X, 1)), Int32(N), mrbo_kernel_id(get_kernel(s)), get_kernel(s).θ[1], s.σn2,
                            fmini, pointer(X), pointer(L), Int32(N), pointer(c), pointer(y),
                            mrbo_kernel_period(get_kernel(s)))
        pd = MrboParamsC(Int32(tp.horizon), Int32(M), Int32(R), Int32(nstarts), mrbo_rule_id(get_decision_rule(s)),
                         θ[1], pointer(lbs), pointer(ubs), Int32(max_iters), Int32(max_ls), 1e-3, 1e-3, 1e-8,
                         1e-4, 1e-8, UInt64(seed), Int32(0), Int32(0), Int32(0), 1.0, Ptr{Float64}(C_NULL))
        mrbo_check(ccall((:mrbo_plan_create, libmrbo), Cint,
                         (Ref{MrboSurrogateC}, Ref{MrboParamsC}, Cint, Ref{Ptr{Cvoid}}), sd, pd, device, h))
    end
    return MrboPlan(h[], size(X, 1), M, R, tp.horizon)
end

# Deterministic release of a plan's device memory (Julia's GC does not see device memory, so no
# finalizer is used: a plan lives until it is destroyed here).  Idempotent.
function mrbo_plan_destroy!(p::MrboPlan)
    if p.handle != C_NULL
        mrbo_check(ccall((:mrbo_plan_destroy, libmrbo), Cint, (Ptr{Cvoid},), p.handle))
        p.handle = C_NULL
    end
    return nothing
end

# ---- plan cache ------------------------------------------------------------------------------
# The reference's outer ascent (stochastic_solve, utils.jl:235-265) calls simulate_trajectory_mc
# up to 50 times per restart on the same surrogate and TrajectoryParameters, moving only x0; a
# plan per call would pack L0⁻¹ on the host, copy the surrogate to HBM and allocate the launch
# workspace every time.  One plan per (surrogate state, tp, θ, start count, M, R, device) is built
# once and reused -- the key holds the surrogate's identity AND a hash of its active data, so a
# conditioned or refitted surrogate gets a new plan.  At most MRBO_PLAN_CACHE_MAX plans live:
# beyond that every cached plan is destroyed (mrbo_plan_destroy!) before the new one is built, and
# mrbo_release_plans!() empties the cache explicitly (also run at exit).
const MRBO_PLAN_CACHE_MAX = 8
const PLAN_CACHE = Dict{Any, MrboPlan}()

function mrbo_release_plans!()
    for p in values(PLAN_CACHE)
        mrbo_plan_destroy!(p)
    end
    empty!(PLAN_CACHE)
    return nothing
end

function mrbo_plan_key(s::Surrogate, tp::TrajectoryParameters, θ::Vector{Float64}, nstarts::Int, device::Int,
                       M::Int, R::Int)
    lbs, ubs = get_spatial_bounds(tp)
    return (objectid(s), get_observed(s), hash(get_active_covariates(s)), hash(get_active_observations(s)),
            hash(get_active_cholesky(s)), hash(get_observations(s)), hash(get_kernel(s).θ), s.σn2,
            get_name(get_decision_rule(s)), tp.horizon, hash(lbs), hash(ubs), θ[1], nstarts, M, R, device)
end

function mrbo_cached_plan(s::Surrogate, tp::TrajectoryParameters, θ::Vector{Float64}, nstarts::Int;
                          device::Int = 0, M::Int = tp.mc_iters, R::Int = 1)
    key = mrbo_plan_key(s, tp, θ, nstarts, device, M, R)
    p = get(PLAN_CACHE, key, nothing)
    p === nothing || return p
    length(PLAN_CACHE) >= MRBO_PLAN_CACHE_MAX && mrbo_release_plans!()
    p = MrboPlan(s, tp, θ, nstarts; device = device, M = M, R = R)
    PLAN_CACHE[key] = p
    return p
end

function __init__()
    atexit(mrbo_release_plans!)
end

# ExpectedTrajectoryOutput tail of rollout.jl:328-339 (the reference's own reductions)
function mrbo_eto(resolutions, gx, gθ)
    μxθ = Distributions.mean(resolutions)
    σ_μxθ = Distributions.std(resolutions, mean=μxθ)
    (isnothing(gx) || isnothing(gθ)) && return ExpectedTrajectoryOutput(μxθ=μxθ, σ_μxθ=σ_μxθ)
    ∇μx = vec(Distributions.mean(gx, dims=2))
    σ_∇μx = vec(Distributions.std(gx, dims=2, mean=∇μx))
    ∇μθ = vec(Distributions.mean(gθ, dims=2))
    σ_∇μθ = vec(Distributions.std(gθ, dims=2, mean=∇μθ))
    return ExpectedTrajectoryOutput(μxθ=μxθ, σ_μxθ=σ_μxθ, ∇μx=∇μx, σ_∇μx=σ_∇μx, ∇μθ=∇μθ, σ_∇μθ=σ_∇μθ)
end

# The GPU method of the reference's simulate_trajectory_mc (rollout.jl:279-340).
function simulate_trajectory_mc(T::Trajectory, tp::TrajectoryParameters, backend::MrboBackend;
                                inner_solve_xstarts::Matrix{Float64}, resolutions::Vector{Float64},
                                spatial_gradients_container::Union{Nothing, Matrix{Float64}} = nothing,
                                hyperparameter_gradients_container::Union{Nothing, Matrix{Float64}} = nothing)
    set_start!(T, get_starting_point(tp))
    plan = mrbo_cached_plan(get_base_surrogate(T), tp, T.θ, size(inner_solve_xstarts, 2); device = backend.device)
    with_grad = !isnothing(spatial_gradients_container) && !isnothing(hyperparameter_gradients_container)
    x0 = copy(T.x0)
    rns = tp.rnstream_sequence
    status = zeros(Int32, tp.mc_iters)
    gx = with_grad ? spatial_gradients_container : Matrix{Float64}(undef, 0, 0)
    gθ = with_grad ? hyperparameter_gradients_container : Matrix{Float64}(undef, 0, 0)
    flags = MRBO_FLAG_HOST_POINTERS | (with_grad ? UInt32(0) : MRBO_FLAG_NO_GRADIENT)
    GC.@preserve x0 rns inner_solve_xstarts resolutions gx gθ status begin
        mrbo_check(ccall((:mrbo_simulate_mc, libmrbo), Cint,
                         (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                          Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Float64}, Ptr{Float64},
                          Ptr{Int64}, UInt32, Ptr{Cvoid}),
                         plan.handle, x0, rns, inner_solve_xstarts, C_NULL, C_NULL, resolutions,
                         with_grad ? pointer(gx) : C_NULL, with_grad ? pointer(gθ) : C_NULL, status,
                         C_NULL, C_NULL, C_NULL, flags, C_NULL))
    end
    any(!=(0), status) && throw(ErrorException("rollout failed on $(count(!=(0), status)) trajectories (status bits $(reduce(|, status)))"))
    return mrbo_eto(resolutions, with_grad ? gx : nothing, with_grad ? gθ : nothing)
end

# Batched restarts: the x0 batch of the outer ascent (generate_batch, utils.jl:97-106) as the
# columns of X0, all of them in ONE launch (R = size(X0, 2) restarts × tp.mc_iters samples on the
# GPU at once; the R = 1 method above puts one x0's 1 024 trajectories on a chip with ≈ 2 048
# resident waves).  Returns one ExpectedTrajectoryOutput per column, each equal to the R = 1
# method's result at that x0 (every trajectory is computed independently of the others in its
# launch; tests/test_gpu.py holds the two call sequences bit for bit).  The optional containers are
# the reference's per restart, stacked: resolutions M×R, spatial gradients d×M×R, hyperparameter
# gradients 1×M×R (overwritten in place).  T is not modified (T.θ is used, Q12).
function simulate_trajectory_mc(T::Trajectory, tp::TrajectoryParameters, X0::Matrix{Float64}, backend::MrboBackend;
                                inner_solve_xstarts::Matrix{Float64}, with_gradient::Bool = true,
                                resolutions::Matrix{Float64} = Matrix{Float64}(undef, tp.mc_iters, size(X0, 2)),
                                spatial_gradients::Union{Nothing, Array{Float64, 3}} = nothing,
                                hyperparameter_gradients::Union{Nothing, Array{Float64, 3}} = nothing)
    d, R = size(X0)
    M = tp.mc_iters
    size(resolutions) == (M, R) || throw(DimensionMismatch("resolutions must be $M×$R"))
    gx = with_grad_container(spatial_gradients, with_gradient, d, M, R)
    gθ = with_grad_container(hyperparameter_gradients, with_gradient, 1, M, R)
    plan = mrbo_cached_plan(get_base_surrogate(T), tp, T.θ, size(inner_solve_xstarts, 2); device = backend.device,
                            R = R)
    rns = tp.rnstream_sequence
    status = zeros(Int32, M, R)
    flags = MRBO_FLAG_HOST_POINTERS | (with_gradient ? UInt32(0) : MRBO_FLAG_NO_GRADIENT)
    GC.@preserve X0 rns inner_solve_xstarts resolutions gx gθ status begin
        mrbo_check(ccall((:mrbo_simulate_mc, libmrbo), Cint,
                         (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                          Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Float64}, Ptr{Float64},
                          Ptr{Int64}, UInt32, Ptr{Cvoid}),
                         plan.handle, X0, rns, inner_solve_xstarts, C_NULL, C_NULL, resolutions,
                         with_gradient ? pointer(gx) : C_NULL, with_gradient ? pointer(gθ) : C_NULL, status,
                         C_NULL, C_NULL, C_NULL, flags, C_NULL))
    end
    any(!=(0), status) && throw(ErrorException("rollout failed on $(count(!=(0), status)) trajectories (status bits $(reduce(|, status)))"))
    return [mrbo_eto(resolutions[:, r], with_gradient ? gx[:, :, r] : nothing, with_gradient ? gθ[:, :, r] : nothing)
            for r in 1:R]
end

with_grad_container(c, with_gradient, a, M, R) =
    !with_gradient ? Array{Float64, 3}(undef, 0, 0, 0) :
    isnothing(c) ? Array{Float64, 3}(undef, a, M, R) :
    size(c) == (a, M, R) ? c : throw(DimensionMismatch("gradient container must be $a×$M×$R"))

# The reference's outer loop on the GPU: stochastic_solve(; optimizer, surrogate, tp, es, start)
# (utils.jl:235-265) for every column of `starts` (d×R, e.g. generate_batch's points, utils.jl:97-106)
# in ONE mrbo_stochastic_solve call on one cached plan: up to `iterations` × [the rollout launch of
# all restarts, their ETO rows, eswavs (utils.jl:114-123) + update! (optimizers.jl)] on the device,
# each restart stopping for good at its eswavs break, with no host round trip per iteration (the
# R = 1 method above, called 50 times per restart by the reference's loop, pays one per call).
# Returns the final points (get_starting_point(tpc) of every restart, d×R) and every restart's ETO
# at its last launch.  θ = tp.θ.  The optimizer's fields are read, never mutated (Adam's moments
# live on the device for the call).
function stochastic_solve(backend::MrboBackend; optimizer::StochasticGradientAscent, surrogate::Surrogate,
                          tp::TrajectoryParameters, es::ExperimentSetup, starts::AbstractMatrix{<:Real},
                          iterations::Int = 50)
    X = Matrix{Float64}(starts)
    d, R = size(X)
    xs = Matrix{Float64}(get_starts(es))
    plan = mrbo_cached_plan(surrogate, tp, tp.θ, size(xs, 2); device = backend.device, R = R)
    rns = tp.rnstream_sequence
    W = 2 + 2d + 2
    eto = Matrix{Float64}(undef, W, R)   # C's R×W rows = the columns here
    active = zeros(Int32, R)
    res = zeros(Int32, 3)
    opts = Ref(mrbo_solve_opts(optimizer, iterations))
    GC.@preserve X rns xs eto active res opts begin
        mrbo_check(ccall((:mrbo_stochastic_solve, libmrbo), Cint,
                         (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ref{MrboSolveOptsC},
                          Ptr{Float64}, Ptr{Int32}, Ptr{Int32}, UInt32, Ptr{Cvoid}),
                         plan.handle, X, rns, xs, C_NULL, opts, eto, active, res, MRBO_FLAG_HOST_POINTERS, C_NULL))
    end
    res[3] != 0 && throw(ErrorException("rollout failed during the ascent (status bits $(res[3]))"))
    etos = [ExpectedTrajectoryOutput(μxθ=eto[1, r], σ_μxθ=eto[2, r], ∇μx=eto[3:2+d, r], σ_∇μx=eto[3+d:2+2d, r],
                                     ∇μθ=eto[3+2d:3+2d, r], σ_∇μθ=eto[4+2d:4+2d, r]) for r in 1:R]
    return X, etos
end

# The GPU method of simulate_trajectory_ghq (rollout.jl:409-467): node vectors nodes[indices[m]]
# and weights[indices[m]] as M×(h+1) matrices for mrbo_simulate_ghq.
function simulate_trajectory_ghq(T::Trajectory, tp::TrajectoryParameters, backend::MrboBackend;
                                 inner_solve_xstarts::Matrix{Float64}, resolutions::Vector{Float64},
                                 nodes::Vector{Float64}, weights::Vector{Float64}, indices,
                                 spatial_gradients_container::Union{Nothing, Matrix{Float64}} = nothing,
                                 hyperparameter_gradients_container::Union{Nothing, Matrix{Float64}} = nothing)
    set_start!(T, get_starting_point(tp))
    M = length(indices)
    depth = length(first(indices))
    tn = Matrix{Float64}(undef, M, depth)
    tw = Matrix{Float64}(undef, M, depth)
    for (m, idx) in enumerate(indices)
        tn[m, :] .= nodes[collect(idx)]
        tw[m, :] .= weights[collect(idx)]
    end
    plan = mrbo_cached_plan(get_base_surrogate(T), tp, T.θ, size(inner_solve_xstarts, 2); device = backend.device,
                            M = M)
    with_grad = !isnothing(spatial_gradients_container) && !isnothing(hyperparameter_gradients_container)
    x0 = copy(T.x0)
    status = zeros(Int32, M)
    gx = with_grad ? spatial_gradients_container : Matrix{Float64}(undef, 0, 0)
    gθ = with_grad ? hyperparameter_gradients_container : Matrix{Float64}(undef, 0, 0)
    flags = MRBO_FLAG_HOST_POINTERS | (with_grad ? UInt32(0) : MRBO_FLAG_NO_GRADIENT)
    GC.@preserve x0 tn tw inner_solve_xstarts resolutions gx gθ status begin
        mrbo_check(ccall((:mrbo_simulate_ghq, libmrbo), Cint,
                         (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                          Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Float64},
                          Ptr{Float64}, Ptr{Int64}, UInt32, Ptr{Cvoid}),
                         plan.handle, x0, tn, tw, inner_solve_xstarts, C_NULL, C_NULL, resolutions,
                         with_grad ? pointer(gx) : C_NULL, with_grad ? pointer(gθ) : C_NULL, status,
                         C_NULL, C_NULL, C_NULL, flags, C_NULL))
    end
    any(!=(0), status) && throw(ErrorException("rollout failed on $(count(!=(0), status)) trajectories"))
    return mrbo_eto(resolutions, with_grad ? gx : nothing, with_grad ? gθ : nothing)
end


# multistart_base_solve!(s::Surrogate, xfinal; spatial_lbs, spatial_ubs, guesses, θfixed)
# (rbf_optim.jl:103-135) with every start's base_solve (:35-66) on the GPU (mrbo_base_solve, one
# wavefront per start, the build's projected Newton in place of IPNewton) and the reference's
# candidate filter and findmin here -- the acquisition step of experiments/myopic_bayesopt.jl.
function mrbo_multistart_base_solve!(s::Surrogate, xfinal::Vector{Float64}; spatial_lbs::Vector{Float64},
                                     spatial_ubs::Vector{Float64}, guesses::Matrix{Float64},
                                     θfixed::Vector{Float64}, device::Int = 0)
    if get_name(get_decision_rule(s)) == "Random"
        xfinal[:] = spatial_lbs .+ (spatial_ubs .- spatial_lbs) .* rand(length(spatial_lbs))
        return nothing
    end
    N = get_observed(s)
    X = Matrix{Float64}(get_active_covariates(s))
    L = Matrix{Float64}(get_active_cholesky(s))
    c = Vector{Float64}(get_active_coefficients(s))
    y = Vector{Float64}(get_active_observations(s))
    d, n = size(guesses)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve X L c y spatial_lbs spatial_ubs begin
        sd = MrboSurrogateC(Int32(d), Int32(N), mrbo_kernel_id(get_kernel(s)), get_kernel(s).θ[1], s.σn2,
                            minimum(get_observations(s)), pointer(X), pointer(L), Int32(N), pointer(c), pointer(y),
                            mrbo_kernel_period(get_kernel(s)))
        pd = MrboParamsC(Int32(0), Int32(1), Int32(1), Int32(1), mrbo_rule_id(get_decision_rule(s)), θfixed[1],
                         pointer(spatial_lbs), pointer(spatial_ubs), Int32(50), Int32(20), 1e-3, 1e-3, 1e-8, 1e-4,
                         1e-8, UInt64(1906), Int32(0), Int32(0), Int32(0), 1.0, Ptr{Float64}(C_NULL))
        mrbo_check(ccall((:mrbo_plan_create, libmrbo), Cint,
                         (Ref{MrboSurrogateC}, Ref{MrboParamsC}, Cint, Ref{Ptr{Cvoid}}), sd, pd, device, h))
    end
    xs, fs, st = zeros(d, n), zeros(n), zeros(Int32, n)
    try
        GC.@preserve guesses xs fs st begin
            mrbo_check(ccall((:mrbo_base_solve, libmrbo), Cint,
                             (Ptr{Cvoid}, Cint, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}, Ptr{Int64},
                              UInt32, Ptr{Cvoid}),
                             h[], n, guesses, xs, fs, st, C_NULL, MRBO_FLAG_HOST_POINTERS, C_NULL))
        end
    finally
        ccall((:mrbo_plan_destroy, libmrbo), Cint, (Ptr{Cvoid},), h[])
    end
    any(!=(0), st) && throw(DomainError(st, "negative posterior variance in base_solve"))
    candidates = [(xs[:, i], fs[i]) for i in 1:n]
    candidates = filter(pair -> !any(isnan.(pair[1])), candidates)       # rbf_optim.jl:129
    mini, j_mini = findmin(pair -> pair[2], candidates)                   # :130
    xfinal .= candidates[j_mini][1]
    return nothing
end


# log_likelihood / ∇log_likelihood (radial_basis_surrogates.jl:770-799) of `s` refit at each
# lengthscale in `ells` on the GPU (mrbo_gp_fit; host arrays, staged by the library).  Returns
# (ll, dll, status) vectors; status 1 marks a PosDefException.  An `optimize!` method can call it
# from its fg! closure (one launch evaluates every trial lengthscale of a line search).
function mrbo_log_likelihood(s::Surrogate, ells::Vector{Float64})
    N = get_observed(s)
    X = Matrix{Float64}(get_active_covariates(s))
    y = Vector{Float64}(get_active_observations(s))
    P = length(ells)
    ll, dll, st = zeros(P), zeros(P), zeros(Int32, P)
    GC.@preserve X y ells ll dll st begin
        sd = MrboSurrogateC(Int32(size(X, 1)), Int32(N), mrbo_kernel_id(get_kernel(s)), get_kernel(s).θ[1], s.σn2,
                            minimum(get_observations(s)), pointer(X), Ptr{Float64}(C_NULL), Int32(N),
                            Ptr{Float64}(C_NULL), pointer(y), mrbo_kernel_period(get_kernel(s)))
        mrbo_check(ccall((:mrbo_gp_fit, libmrbo), Cint,
                         (Ref{MrboSurrogateC}, Cint, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32},
                          Ptr{Float64}, Ptr{Float64}, UInt32, Ptr{Cvoid}),
                         sd, P, ells, ll, dll, st, C_NULL, C_NULL, MRBO_FLAG_HOST_POINTERS, C_NULL))
    end
    return ll, dll, st
end

end # module
