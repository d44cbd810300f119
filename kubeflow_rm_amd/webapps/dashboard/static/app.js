// Central dashboard shell: menu from /api/dashboard-links, namespace selector from the user's
// workgroups (/api/workgroup/env-info), iframe container for the apps under /_/<app>/ speaking the
// library.js protocol, home page (quick links, activities, resource + MI355X GPU allocation charts),
// registration flow and contributor management.
(function () {
  "use strict";
  const $ = (id) => document.getElementById(id);
  const state = { env: null, links: {}, ns: localStorage.getItem("kf-namespace") || "", frame: null };
  const esc = (s) => String(s == null ? "" : s).replace(/[&<>"]/g, (c) => ({ "&": "&amp;", "<": "&lt;", ">": "&gt;", '"': "&quot;" }[c]));
  async function get(path) { const r = await fetch(path); const d = await r.json(); if (!r.ok) throw new Error(d.error || r.statusText); return d; }
  async function send(method, path, body) {
    const r = await fetch(path, { method, headers: { "Content-Type": "application/json" }, body: JSON.stringify(body || {}) });
    const d = await r.json(); if (!r.ok) throw new Error(d.error || r.statusText); return d;
  }

  function postNamespace() {
    if (!state.frame || !state.frame.contentWindow) return;
    state.frame.contentWindow.postMessage({ type: "namespace-selected", value: state.ns }, "*");
  }
  window.addEventListener("message", (ev) => {
    if ((ev.data || {}).type === "iframe-connected") postNamespace();
  });

  function renderMenu() {
    const items = (state.links.menuLinks || []).map((l) => `<a href="/_${esc(l.link)}" data-link="${esc(l.link)}">${esc(l.text)}</a>`);
    const ext = (state.links.externalLinks || []).map((l) => `<a href="${esc(l.link)}" target="_blank">${esc(l.text)} &#8599;</a>`);
    $("menu").innerHTML = `<a href="/" data-link="/">Home</a>${items.join("")}<a href="/manage-users" data-link="/manage-users">Manage contributors</a>` +
      (ext.length ? `<h4>External</h4>${ext.join("")}` : "");
    $("menu").querySelectorAll("a[data-link]").forEach((a) => a.addEventListener("click", (e) => { e.preventDefault(); navigate(a.getAttribute("href")); }));
  }

  function renderNamespaces() {
    const nss = (state.env.namespaces || []).map((b) => b.namespace);
    if (!nss.includes(state.ns)) state.ns = nss[0] || "";
    $("ns").innerHTML = nss.map((n) => `<option ${n === state.ns ? "selected" : ""}>${esc(n)}</option>`).join("");
    $("ns").onchange = () => { state.ns = $("ns").value; localStorage.setItem("kf-namespace", state.ns); postNamespace(); route(); };
  }

  function navigate(href) { history.pushState({}, "", href); route(); }
  window.addEventListener("popstate", route);

  function route() {
    const p = location.pathname;
    $("menu").querySelectorAll("a[data-link]").forEach((a) => a.classList.toggle("active", p === a.getAttribute("href")));
    if (p.startsWith("/_/")) return showIframe(p.slice(2) + location.search);
    if (p === "/manage-users") return showManageUsers();
    return showHome();
  }

  function showIframe(src) {
    const sep = src.includes("?") ? "&" : "?";
    $("content").innerHTML = "";
    state.frame = document.createElement("iframe");
    state.frame.src = src + (state.ns ? `${sep}ns=${encodeURIComponent(state.ns)}` : "");
    state.frame.addEventListener("load", () => state.frame.contentWindow.postMessage({ type: "parent-connected" }, "*"));
    $("content").append(state.frame);
  }

  function chart(points, title) {
    if (!points.length) return `<p>${esc(title)}: no data</p>`;
    const w = 300, h = 80, t0 = points[0].timestamp, t1 = points[points.length - 1].timestamp || t0 + 1;
    const vmax = Math.max(1e-9, ...points.map((p) => p.value));
    const path = points.map((p, i) => `${i ? "L" : "M"}${((p.timestamp - t0) / Math.max(1, t1 - t0)) * w},${h - (p.value / vmax) * h}`).join(" ");
    return `<div>${esc(title)} <small>(max ${(vmax * 100).toFixed(1)})</small><br><svg width="${w}" height="${h}"><path d="${path}" fill="none" stroke="#1a73e8"/></svg></div>`;
  }

  async function showHome() {
    state.frame = null;
    const quick = (state.links.quickLinks || []).map((l) => `<li><a href="/_${esc(l.link)}">${esc(l.text)}</a> <small>${esc(l.desc || "")}</small></li>`).join("");
    const docs = (state.links.documentationItems || []).map((l) => `<li><a href="${esc(l.link)}" target="_blank">${esc(l.text)}</a></li>`).join("");
    $("content").innerHTML = `<div class="page"><div class="cards">
      <div class="card"><h3>Quick shortcuts</h3><ul>${quick}</ul></div>
      <div class="card"><h3>Recent notebooks in ${esc(state.ns)}</h3><div id="nbs">loading…</div></div>
      <div class="card"><h3>Recent activity in ${esc(state.ns)}</h3><div id="acts">loading…</div></div>
      <div class="card"><h3>Cluster resources</h3><div id="charts">loading…</div></div>
      <div class="card"><h3>Documentation</h3><ul>${docs}</ul></div></div></div>`;
    if (state.ns) {
      get(`/jupyter/api/namespaces/${encodeURIComponent(state.ns)}/notebooks`).then((d) => {
        const nbs = (d.notebooks || []).slice(0, 5);
        $("nbs").innerHTML = nbs.map((nb) => `<div><a href="/notebook/${esc(state.ns)}/${esc(nb.name)}/" target="_blank">${esc(nb.name)}</a>
          <small>${esc(nb.status.phase)} · ${esc(nb.gpus.message || "no GPU")}</small></div>`).join("") || "none";
      }).catch(() => { $("nbs").textContent = "Notebooks app unavailable"; });
      get(`/api/activities/${encodeURIComponent(state.ns)}`).then((evs) => {
        evs.sort((a, b) => String(b.lastTimestamp || b.metadata.creationTimestamp).localeCompare(String(a.lastTimestamp || a.metadata.creationTimestamp)));
        $("acts").innerHTML = `<table>${evs.slice(0, 20).map((e) => `<tr><td>${esc(e.lastTimestamp || e.metadata.creationTimestamp)}</td><td>${esc(e.involvedObject.kind)}/${esc(e.involvedObject.name)}</td><td>${esc(e.message)}</td></tr>`).join("")}</table>` || "none";
      }).catch((e) => { $("acts").textContent = e.message; });
    }
    Promise.all(["node", "podcpu", "gpu"].map((k) => get(`/api/metrics/${k}?interval=Last60m`).catch(() => null))).then(([n, c, g]) => {
      if (!n) { $("charts").textContent = "Metrics are not available on this cluster."; return; }
      $("charts").innerHTML = chart(n, "Node CPU") + chart(c || [], "Pod CPU requests") + chart(g || [], "MI355X GPUs allocated");
    });
  }

  async function showManageUsers() {
    state.frame = null;
    const owned = (state.env.namespaces || []).filter((b) => b.role === "owner");
    $("content").innerHTML = `<div class="page"><h2>Manage contributors</h2><p class="err" id="merr"></p>${owned.map((b) => `
      <div class="card"><h3>${esc(b.namespace)}</h3><div id="c-${esc(b.namespace)}">loading…</div>
      <input id="i-${esc(b.namespace)}" placeholder="user@example.com"> <button data-ns="${esc(b.namespace)}">Add</button></div>`).join("") || "<p>You do not own a namespace.</p>"}</div>`;
    const render = (ns, users) => {
      $(`c-${ns}`).innerHTML = users.map((u) => `${esc(u)} <button data-rm="${esc(u)}" data-ns="${esc(ns)}">remove</button>`).join("<br>") || "no contributors";
      $(`c-${ns}`).querySelectorAll("button[data-rm]").forEach((btn) => btn.onclick = () =>
        send("DELETE", `/api/workgroup/remove-contributor/${ns}`, { contributor: btn.dataset.rm }).then((u) => render(ns, u)).catch((e) => { $("merr").textContent = e.message; }));
    };
    owned.forEach((b) => get(`/api/workgroup/get-contributors/${b.namespace}`).then((u) => render(b.namespace, u)).catch((e) => { $("merr").textContent = e.message; }));
    $("content").querySelectorAll("button[data-ns]:not([data-rm])").forEach((btn) => btn.onclick = () => {
      const ns = btn.dataset.ns;
      send("POST", `/api/workgroup/add-contributor/${ns}`, { contributor: $(`i-${ns}`).value }).then((u) => render(ns, u)).catch((e) => { $("merr").textContent = e.message; });
    });
  }

  function showRegistration(ex) {
    $("menu").innerHTML = "";
    $("content").innerHTML = `<div class="page"><h2>Welcome, ${esc(ex.user)}</h2><p>Create your namespace to start using notebooks on MI355X GPUs.</p>
      <input id="reg-ns" value="${esc(ex.user)}"> <button id="reg">Finish</button> <span class="err" id="rerr"></span></div>`;
    $("reg").onclick = () => send("POST", "/api/workgroup/create", { namespace: $("reg-ns").value })
      .then(() => setTimeout(main, 1000)).catch((e) => { $("rerr").textContent = e.message; });
  }

  async function main() {
    try {
      const ex = await get("/api/workgroup/exists");
      if (ex.hasAuth && !ex.hasWorkgroup && ex.registrationFlowAllowed) return showRegistration(ex);
      [state.env, state.links] = await Promise.all([get("/api/workgroup/env-info"), get("/api/dashboard-links").catch(() => ({}))]);
      $("user").textContent = state.env.user;
      $("logout").href = (state.env.platform || {}).logoutUrl || "/logout";
      renderMenu(); renderNamespaces(); route();
    } catch (e) { $("content").innerHTML = `<p class="page err">${esc(e.message)}</p>`; }
  }
  main();
})();
