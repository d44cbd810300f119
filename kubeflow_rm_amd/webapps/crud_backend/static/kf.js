// kf.js — shared frontend runtime of the CRUD apps (the kubeflow-common-lib role, vanilla JS):
// backend calls with the CSRF double-submit header, exponential-backoff poller (1 s -> 8 s, reset
// when the data changes), namespace selection bound to the central dashboard's iframe protocol
// (library.js: parent-connected / iframe-connected / namespace-selected / all-namespaces), status
// icons and small DOM helpers.
(function (global) {
  "use strict";
  function cookie(name) {
    const m = document.cookie.match(new RegExp("(?:^|; )" + name.replace(/[-.]/g, "\\$&") + "=([^;]*)"));
    return m ? decodeURIComponent(m[1]) : "";
  }
  async function call(method, path, body) {
    const opts = { method, headers: { "Accept": "application/json" }, credentials: "same-origin" };
    if (method !== "GET") opts.headers["X-XSRF-TOKEN"] = cookie("XSRF-TOKEN");
    if (body !== undefined) {
      opts.headers["Content-Type"] = "application/json";
      opts.body = JSON.stringify(body);
    }
    const r = await fetch(path.replace(/^\//, ""), opts);
    let data = {};
    try { data = await r.json(); } catch (e) { data = { success: false, log: r.statusText }; }
    if (!r.ok || data.success === false) throw new Error(data.log || r.statusText);
    return data;
  }
  class Poller {
    constructor(fn, min = 1000, max = 8000) { this.fn = fn; this.min = min; this.max = max; this.delay = min; this.last = null; this.t = null; }
    start() { this.stop(); this.tick(); return this; }
    stop() { if (this.t) clearTimeout(this.t); this.t = null; }
    reset() { this.delay = this.min; this.start(); }
    async tick() {
      let sig = null;
      try { sig = JSON.stringify(await this.fn()); } catch (e) { console.warn(e); }
      if (sig !== null && sig !== this.last) { this.delay = this.min; this.last = sig; }
      else this.delay = Math.min(this.delay * 2, this.max);
      this.t = setTimeout(() => this.tick(), this.delay);
    }
  }
  // namespace service: inside the dashboard iframe the parent drives the selection
  const nsListeners = [];
  let currentNs = new URLSearchParams(location.search).get("ns") || localStorage.getItem("kf-namespace") || "";
  function setNamespace(ns) {
    if (!ns || ns === currentNs) return;
    currentNs = ns;
    localStorage.setItem("kf-namespace", ns);
    nsListeners.forEach((f) => f(ns));
  }
  function onNamespace(f) { nsListeners.push(f); if (currentNs) f(currentNs); }
  window.addEventListener("message", (ev) => {
    const d = ev.data || {};
    if (d.type === "namespace-selected" && d.value) setNamespace(d.value);
    if (d.type === "parent-connected" && window.parent !== window) window.parent.postMessage({ type: "iframe-connected" }, "*");
  });
  if (window.parent !== window) window.parent.postMessage({ type: "iframe-connected" }, "*");
  const icons = { ready: "&#9679;", waiting: "&#9676;", warning: "&#9888;", error: "&#10006;", stopped: "&#9632;",
                  terminating: "&#8987;", unavailable: "&#8709;", uninitialized: "&#9675;" };
  function statusCell(st) {
    st = st || {};
    return `<span class="st st-${st.phase}" title="${(st.message || "").replace(/"/g, "&quot;")}">${icons[st.phase] || "?"} ${st.phase || ""}</span>`;
  }
  function h(tag, attrs, ...children) {
    const e = document.createElement(tag);
    Object.entries(attrs || {}).forEach(([k, v]) => (k.startsWith("on") ? e.addEventListener(k.slice(2), v) : e.setAttribute(k, v)));
    children.flat().forEach((c) => e.append(c instanceof Node ? c : document.createTextNode(String(c))));
    return e;
  }
  global.kf = { call, Poller, cookie, setNamespace, onNamespace, namespace: () => currentNs, statusCell, h };
})(window);
