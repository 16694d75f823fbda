// penroz dashboard: polls /progress and /stats and draws them on plain <canvas> elements
// (no third-party charting library).

const PALETTE = ["#1f77b4", "#ff7f0e", "#2ca02c", "#d62728", "#9467bd", "#8c564b", "#e377c2",
                 "#7f7f7f", "#bcbd22", "#17becf"];

function el(tag, attrs = {}, text = "") {
  const e = document.createElement(tag);
  for (const [k, v] of Object.entries(attrs)) e.setAttribute(k, v);
  if (text) e.textContent = text;
  return e;
}

function card(title, w = 460, h = 240) {
  const c = el("div", { class: "card" });
  c.appendChild(el("h3", {}, title));
  const cv = el("canvas", { width: w, height: h });
  c.appendChild(cv);
  document.getElementById("charts").appendChild(c);
  return cv;
}

function bounds(series) {
  let xmin = Infinity, xmax = -Infinity, ymin = Infinity, ymax = -Infinity;
  for (const s of series) for (const [x, y] of s.points) {
    if (y === null || !isFinite(y)) continue;
    xmin = Math.min(xmin, x); xmax = Math.max(xmax, x);
    ymin = Math.min(ymin, y); ymax = Math.max(ymax, y);
  }
  if (!isFinite(xmin)) return null;
  if (xmax === xmin) xmax = xmin + 1;
  if (ymax === ymin) { ymax += 0.5; ymin -= 0.5; }
  return { xmin, xmax, ymin, ymax };
}

// series: [{label, points: [[x, y], ...]}]; kind: "line" | "bars"
function plot(canvas, series, kind = "line", logY = false) {
  const ctx = canvas.getContext("2d");
  const W = canvas.width, H = canvas.height, L = 52, R = 8, T = 8, B = 34;
  ctx.clearRect(0, 0, W, H);
  const tr = v => (logY ? Math.log10(Math.max(v, 1e-12)) : v);
  const s2 = series.map(s => ({ ...s, points: s.points.filter(p => p[1] !== null).map(([x, y]) => [x, tr(y)]) }));
  const b = bounds(s2);
  if (!b) { ctx.fillText("no data", W / 2 - 20, H / 2); return; }
  const X = x => L + (x - b.xmin) / (b.xmax - b.xmin) * (W - L - R);
  const Y = y => T + (1 - (y - b.ymin) / (b.ymax - b.ymin)) * (H - T - B);
  ctx.strokeStyle = "#999"; ctx.lineWidth = 1;
  ctx.beginPath(); ctx.moveTo(L, T); ctx.lineTo(L, H - B); ctx.lineTo(W - R, H - B); ctx.stroke();
  ctx.fillStyle = "#444"; ctx.font = "10px sans-serif";
  for (let i = 0; i <= 4; i++) {
    const yv = b.ymin + (b.ymax - b.ymin) * i / 4;
    ctx.fillText((logY ? "1e" + yv.toFixed(1) : yv.toPrecision(3)), 2, Y(yv) + 3);
    const xv = b.xmin + (b.xmax - b.xmin) * i / 4;
    ctx.fillText(xv.toPrecision(3), X(xv) - 10, H - B + 12);
  }
  s2.forEach((s, i) => {
    ctx.strokeStyle = ctx.fillStyle = PALETTE[i % PALETTE.length];
    if (kind === "bars") {
      const w = Math.max(1, (W - L - R) / Math.max(1, s.points.length) * 0.9);
      for (const [x, y] of s.points) ctx.fillRect(X(x), Y(y), w, H - B - Y(y));
    } else {
      ctx.beginPath();
      s.points.forEach(([x, y], j) => (j ? ctx.lineTo(X(x), Y(y)) : ctx.moveTo(X(x), Y(y))));
      ctx.stroke();
    }
  });
  ctx.font = "10px sans-serif";
  s2.slice(0, 8).forEach((s, i) => {
    ctx.fillStyle = PALETTE[i % PALETTE.length];
    ctx.fillText(s.label, L + 6 + (i % 4) * 100, H - 6 - Math.floor(i / 4) * 11);
  });
}

function layerSelected(filter, algo, idx) {
  if (!filter.trim()) return true;
  return filter.split(",").map(t => t.trim().toLowerCase()).some(t => t === String(idx) || algo.includes(t));
}

async function refresh() {
  const id = document.getElementById("model-id").value.trim();
  const filter = document.getElementById("layer-filter").value;
  const status = document.getElementById("status");
  const charts = document.getElementById("charts");
  if (!id) { status.textContent = "enter a model id"; return; }
  charts.innerHTML = "";
  let prog;
  try {
    const r = await fetch(`/progress/?model_id=${encodeURIComponent(id)}`);
    if (!r.ok) { status.textContent = `progress: HTTP ${r.status}`; return; }
    prog = await r.json();
  } catch (e) { status.textContent = "progress request failed: " + e; return; }
  const st = prog.status || {};
  const last = (prog.progress || []).slice(-1)[0];
  status.textContent = `${st.code || "?"} — ${st.message || ""} ${st.dt || ""}` +
    (last ? ` | epoch ${last.epoch} cost ${last.cost.toFixed(4)} | ${Math.round(last.tokensPerSec || last.speedPerSec)} tok/s` : "");

  const progress = prog.progress || [];
  plot(card("cost per epoch"), [{ label: "cost", points: progress.map(p => [p.epoch, p.cost]) }]);
  plot(card("average cost history"), [{ label: "avg cost", points: (prog.average_cost_history || []).map((c, i) => [i, c]) }]);
  plot(card("throughput (tokens/s)"), [
    { label: "whole job", points: progress.map(p => [p.epoch, p.tokensPerSec || null]) },
    { label: "speedPerSec", points: progress.map(p => [p.epoch, p.speedPerSec]) }]);
  const nW = progress.length ? (progress[0].weight_upd_ratio || []).length : 0;
  const upd = [];
  for (let w = 0; w < nW; w++) {
    const pts = progress.map(p => [p.epoch, p.weight_upd_ratio[w]]).filter(p => p[1] !== null);
    if (pts.length) upd.push({ label: `w${w}`, points: pts });
  }
  plot(card("weight update ratio (log10)"), upd, "line", true);

  let stats = null;
  try {
    const r = await fetch(`/stats/?model_id=${encodeURIComponent(id)}`);
    if (r.ok) stats = await r.json();
  } catch (e) { /* stats are optional */ }
  if (!stats) return;
  const acts = [], grads = [], sat = [];
  (stats.layers || []).forEach((l, i) => {
    if (!layerSelected(filter, l.algo, i)) return;
    const label = `${i}:${l.algo}`;
    acts.push({ label, points: l.activation.histogram.x.map((x, j) => [x, l.activation.histogram.y[j]]) });
    sat.push({ label, points: [[i, l.activation.saturated]] });
    if (l.gradient) grads.push({ label, points: l.gradient.histogram.x.map((x, j) => [x, l.gradient.histogram.y[j]]) });
  });
  plot(card("activation distributions"), acts);
  plot(card("activation gradient distributions"), grads);
  plot(card("saturation by layer"), sat, "bars");
  const wg = [];
  (stats.weights || []).forEach((w, i) => {
    if (!w || !w.gradient || !w.gradient.histogram.x.length) return;
    wg.push({ label: `w${i} ${w.shape}`, points: w.gradient.histogram.x.map((x, j) => [x, w.gradient.histogram.y[j]]) });
  });
  plot(card("weight gradient distributions"), wg);
}

let timer = null;
window.addEventListener("load", () => {
  document.getElementById("refresh").addEventListener("click", refresh);
  document.getElementById("auto").addEventListener("change", e => {
    if (timer) clearInterval(timer);
    timer = e.target.checked ? setInterval(refresh, 5000) : null;
  });
  const q = new URLSearchParams(location.search).get("model_id");
  if (q) { document.getElementById("model-id").value = q; refresh(); }
});
